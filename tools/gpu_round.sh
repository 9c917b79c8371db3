#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/abort/timeout (exit status
# other than 0 or 1) ends the script so nothing else touches the GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export MP_LOG_DIR=gpurun_out/mp
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    echo "== $name: $*" | tee -a gpurun_out/steps.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
    tail -5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
for s in ${STEPS:-smoke tests bench prof}; do
  case $s in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${KEXPR:+-k "$KEXPR"} ${PYTEST_ARGS} ;;
    ldpre) OSGPU_LIB_PATH=tools/ldvariant/libosgpu_pre.so step ldpre 300 python -u tools/ld_team_rate.py ;;
    ldtest) step ldtest 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py ;;
    ldrate) step ldrate 300 python -u tools/ld_team_rate.py &&
            TR_TYPE=longdouble step ldcall 300 python -u tools/team_rate.py $((8<<20)) ;;
    ldpmc3) LD_ONLY=sum/random/8 REPS=5 step ldpmc_r 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -d gpurun_out/ldpmc_r -o run --output-format csv -- python3 tools/ld_team_rate.py &&
            LD_ONLY=sum/positive/8 REPS=5 step ldpmc_p 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -d gpurun_out/ldpmc_p -o run --output-format csv -- python3 tools/ld_team_rate.py &&
            LD_ONLY=sum/ones/8 REPS=5 step ldpmc_o 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -d gpurun_out/ldpmc_o -o run --output-format csv -- python3 tools/ld_team_rate.py ;;
    ldpmc) export LD_ONLY=sum/random/8 REPS=5
           step ldpmc1 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/ldpmc1 -o run --output-format csv -- python3 tools/ld_team_rate.py &&
           step ldpmc2 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/ldpmc2 -o run --output-format csv -- python3 tools/ld_team_rate.py ;;
    xover) step xover 600 python -u tools/crossover.py ;;
    nsprobe) step nsprobe 300 python -u tools/ns_probe.py ${NS_ARGS} ;;
    vmmprobe) step vmmprobe 200 python -u tools/vmm_probe.py 2 ;;
    vmm)   step vmm 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_multiproc.py -k vmm ;;
    bench) step bench 600 python bench.py ${BENCH_ARGS} ;;
    prof)  step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-live-pmc --no-cpu-baseline --no-api --no-extra --steps 20 --warmup 5 ;;
    tune)  step tune 300 ./tools/tune_combine ;;
    tunens) step tunens${TUNE_N}a${ALLOC}c${CHUNK} 300 ./tools/tune_ns ${TUNE_N:-134217728} ${TUNE_REPS:-20} ;;
    latency) step latency 300 python tools/latency_probe.py ;;
    mplat) step mplat 400 python tools/mp_latency.py ;;
    multi) step multi2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --nreduce $((64<<20)) --c4-nreduce $((256<<20)) --c5-nreduce $((64<<20)) --deadline 200 ;;
    multi_s) step multi2 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --nreduce $((4<<20)) --c4-nreduce $((8<<20)) --c5-nreduce $((4<<20)) --deadline 120 ;;
    r3tests) step r3tests 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_multiproc.py -k "preflight or mixed_topology or heap_reuse" ;;
    multi_self) step multi_self 420 python bench.py --gpus 2 --steps 5 --warmup 2 --deadline 360 ;;
    multi_self4) step multi_self4 420 python bench.py --gpus 4 --steps 3 --warmup 1 --nreduce $((16<<20)) --c4-nreduce $((64<<20)) --c5-nreduce $((16<<20)) --deadline 360 ;;
    multi_tr2) step multi_tr2 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29515 bench.py --gpus 2 --steps 5 --warmup 2 --deadline 360 ;;
    multi8) step multi8 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 8 --steps 5 --warmup 2 --deadline 800 ;;
    teamlayout) step teamlayout 300 python -u tools/team_layout_probe.py && TL_P=2 step teamlayout2 300 python -u tools/team_layout_probe.py && TL_P=8 TL_N=$((32<<20)) step teamlayout8 300 python -u tools/team_layout_probe.py ;;
    copyvar) step copyvar 600 python -u tools/team_variants.py run_copy ;;
    teamvar) step teamvar 900 python -u tools/team_variants.py run ;;
    sweep) step sweep 900 python -u tools/team_variants.py run_sweep ;;
    place) step place 600 python -u tools/team_variants.py run_place ;;
    ldprof) step ldprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ldprof -o run --output-format csv -- python3 tools/ld_rocprof.py run &&
            python3 tools/ld_rocprof.py parse gpurun_out/ldprof gpurun_out/ldprof.log gpurun_out/ld_rocprof.json ;;
    callov) step callov 600 python -u tools/call_overhead.py ;;
    smallenv) step smallenv 600 python -u tools/small_call_env.py ;;
    teamtlb) step teamtlb 300 rocprofv3 --pmc TCP_UTCL1_REQUEST TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_THRASHING_STALL -d gpurun_out/teamtlb -o run --output-format csv -- python3 tools/team_tlb_probe.py run &&
             python3 tools/team_tlb_probe.py parse gpurun_out/teamtlb gpurun_out/teamtlb.log gpurun_out/team_tlb.jsonl ;;
    teamea) export TT_COUNTERS=TCC_EA0_RDREQ,TCC_EA0_WRREQ
            step counters 120 rocprofv3 --list-avail &&
            step teamea 300 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_WRREQ -d gpurun_out/teamea -o run --output-format csv -- python3 tools/team_tlb_probe.py run &&
            python3 tools/team_tlb_probe.py parse gpurun_out/teamea gpurun_out/teamea.log gpurun_out/team_ea.jsonl ;;
    teamstall) export TT_COUNTERS=TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum,TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum,TCC_EA0_WRREQ_STALL_sum,TCC_TOO_MANY_EA_WRREQS_STALL_sum
            step teamstall 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum -d gpurun_out/teamstall -o run --output-format csv -- python3 tools/team_tlb_probe.py run &&
            python3 tools/team_tlb_probe.py parse gpurun_out/teamstall gpurun_out/teamstall.log gpurun_out/team_stall.jsonl ;;
    tuneteam) step tuneteam 400 ./tools/tune_team ;;
    teamlayouts) step teamlayouts 400 ./tools/tune_team $((64<<20)) 20 6 layouts ;;
    teamoff) step teamoff 300 python -u tools/team_offsets.py ;;
    multi8_small) step multi8_small 600 python bench.py --gpus 8 --steps 3 --warmup 1 --nreduce $((16<<20)) --c4-nreduce $((64<<20)) --c5-nreduce $((16<<20)) --deadline 500 ;;
    multi8_self) step multi8_self 900 python bench.py --gpus 8 --steps 5 --warmup 2 --deadline 800 ;;
    multi4_s) step multi4 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 4 --steps 3 --warmup 1 --nreduce $((4<<20)) --c4-nreduce $((8<<20)) --c5-nreduce $((4<<20)) --deadline 200 ;;
    proffull) step proffull 900 rocprofv3 --kernel-trace --stats -d gpurun_out/proffull -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    prof3) step prof3 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python3 bench.py --no-live-pmc --no-cpu-baseline --no-api --steps 20 --warmup 5 ;;
    pmc3)  step pmc3f 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc3f -o run --output-format csv -- python3 bench.py --no-live-pmc --no-cpu-baseline --no-api --steps 5 --warmup 2 &&
           step pmc3w 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc3w -o run --output-format csv -- python3 bench.py --no-live-pmc --no-cpu-baseline --no-api --steps 5 --warmup 2 &&
           python3 tools/pmc_traffic.py gpurun_out/pmc3f gpurun_out/pmc3w $((64<<20)) gpurun_out/traffic.json &&
           python3 tools/pmc_traffic.py gpurun_out/pmc3f gpurun_out/pmc3w $((64<<20)) gpurun_out/traffic_team.json "team_vec_kernel<double, 0, 2, true>" 32 &&
           python3 tools/pmc_traffic.py gpurun_out/pmc3f gpurun_out/pmc3w $((64<<20)) gpurun_out/traffic_team4.json "team_lds_kernel<double, 0, 4, true, 4" 64 &&
           python3 tools/pmc_traffic.py gpurun_out/pmc3f gpurun_out/pmc3w $((64<<20)) gpurun_out/traffic_team8.json "team_vec_kernel<double, 0, 8, true>" 128 ;;
    pmc)   step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --no-live-pmc --no-cpu-baseline --no-api --no-extra --steps 5 --warmup 2 &&
           step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --no-live-pmc --no-cpu-baseline --no-api --no-extra --steps 5 --warmup 2 &&
           python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write $((64<<20)) gpurun_out/traffic.json &&
           python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write $((64<<20)) gpurun_out/traffic_team.json "team_vec_kernel<double, 0, 2, true>" 32 ;;
  esac
done
echo "all steps done"
