mkdir -p gpurun_out
export SWEEP_SETTINGS='[{}, {"OSGPU_COPY_THREADS_TOTAL": "0"}, {"OSGPU_COPY_THREADS_TOTAL": "4"}, {"OSGPU_COPY_THREADS_TOTAL": "16"}, {"OSGPU_HOST_BOUNCE": "0"}]'
SWEEP_PES=4 timeout -k 10 400 python tools/sweep_host_staged.py > gpurun_out/sw4.jsonl 2>&1 && SWEEP_PES=2 timeout -k 10 300 python tools/sweep_host_staged.py > gpurun_out/sw2.jsonl 2>&1
