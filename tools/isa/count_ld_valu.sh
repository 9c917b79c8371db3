#!/bin/bash
# Static VALU count of the long double team sum at P = 8 for a given x87.hpp:
#   tools/isa/count_ld_valu.sh [path/to/x87.hpp]   (default: the shipped one)
# compiles tools/isa/ld_team_sum8.hip (the ld_team_kernel loop body) for
# gfx950 and prints the VALU / SALU / s_nop count of every straight-line
# round of 7 soft adds (tools/isa/count_rounds.py).  Not part of the product.
here=$(cd "$(dirname "$0")" && pwd)
hpp=${1:-$here/../../test-resilient-osss-ucx_amd/csrc/x87.hpp}
d=$(mktemp -d); cp "$hpp" $d/x87.hpp; cp $here/ld_team_sum8.hip $d/ldk.hip
cd $d && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math --save-temps -c ldk.hip -o ldk.o 2>&1 | grep -i error
awk '/^_Z3ldkILi0ELi8EEv6LdTeamm:/,/s_endpgm/' ldk-hip-amdgcn-amd-amdhsa-gfx950.s > k.s
python3 $here/count_rounds.py k.s
rm -rf $d
