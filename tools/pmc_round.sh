#!/bin/bash
# PMC traffic files for the shipped kernels (FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 passes over tools/pmc_probe.py), written to
# gpurun_out/traffic/*.json by tools/pmc_traffic.py.  Not product.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/traffic; mkdir -p $O
N=$((64<<20))
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/F -o run --output-format csv -- python3 tools/pmc_probe.py $N 5 2 4 8 > $O/F.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/W -o run --output-format csv -- python3 tools/pmc_probe.py $N 5 2 4 8 > $O/W.log 2>&1
python3 tools/pmc_traffic.py $O/F $O/W $N $O/r05_traffic.json "combine_lds_kernel<double, 0, 2, 2>" 24
python3 tools/pmc_traffic.py $O/F $O/W $N $O/r05_traffic_team2.json "team_lds_kernel<double, 0, 2, true, 2" 32
python3 tools/pmc_traffic.py $O/F $O/W $N $O/r05_traffic_team4.json "team_lds_kernel<double, 0, 4, true, 2" 64
python3 tools/pmc_traffic.py $O/F $O/W $N $O/r05_traffic_team8.json "team_vec_kernel<double, 0, 8, true>" 128
rm -rf $O/F $O/W
