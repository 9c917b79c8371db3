"""Register budget of every kernel in the built library, read from the
gfx950 code objects' metadata (no GPU needed): the .hip_fatbin section of
each in-tree object (csrc/*.o), unbundled with clang-offload-bundler, its
notes read with llvm-readelf, parsed by tools/isa/reg_table.py.

* no kernel uses AGPRs (the accumulation registers are MFMA state; none of
  these kernels multiplies matrices -- an AGPR here is a spill in disguise);
* every kernel keeps at least 2 waves per SIMD, every team kernel at least 3
  (complexf prod at 8 members ran at 1 wave with 276 VGPRs +
  20 AGPRs; now 134 VGPRs, 3 waves, the only team kernel above 128);
* no scratch, except the x87 long double 7- and 8-member sum team kernels
  (at most 64 B per lane; today 0 / 48 B, 9 spilled VGPRs at 8 members,
  128 VGPRs, 4 waves per SIMD: the trade of x87.hpp fold_rounds, whose two
  groups of folds took the 8-member sum from 57 spilled VGPRs to 10, the
  sign mask and the near rounds' dropped terms to 9).

Skipped when the objects or the LLVM tools are absent (e.g. on the GPU box,
where only the linked library travels).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "test-resilient-osss-ucx_amd", "csrc")
LLVM = "/opt/rocm/lib/llvm/bin"
OBJS = ("combine", "team", "fused", "verify", "longdouble", "copy")
sys.path.insert(0, os.path.join(ROOT, "tools", "isa"))


def _kernels(obj, tmp):
    o = os.path.join(CSRC, obj + ".o")
    fat, co, notes = (os.path.join(tmp, obj + s) for s in (".fat", ".co", ".notes"))
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", o,
                    os.path.join(tmp, obj + ".stripped")], check=True, capture_output=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                    f"--input={fat}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                    f"--output={co}"], check=True, capture_output=True)
    with open(notes, "w") as f:
        subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True, stdout=f)
    import reg_table
    return reg_table.parse(notes)


@pytest.fixture(scope="module")
def kernels(tmp_path_factory):
    if not all(os.path.exists(os.path.join(CSRC, o + ".o")) for o in OBJS):
        pytest.skip("in-tree objects absent (build() not run here)")
    if not os.path.exists(os.path.join(LLVM, "clang-offload-bundler")):
        pytest.skip("LLVM offload tools absent")
    tmp = str(tmp_path_factory.mktemp("isa"))
    return {o: _kernels(o, tmp) for o in OBJS}


def test_every_object_has_kernels(kernels):
    for o, rows in kernels.items():
        assert rows, o


def test_no_agprs_and_at_least_two_waves(kernels):
    bad = [(o, r["kernel"][:100], r["vgpr"], r["agpr"], r["waves_per_simd"])
           for o, rows in kernels.items() for r in rows
           if r["agpr"] > 0 or r["waves_per_simd"] < 2]
    assert not bad, json.dumps(bad[:10])


def test_team_kernels_keep_three_waves(kernels):
    bad = [(r["kernel"][:100], r["vgpr"], r["waves_per_simd"]) for r in kernels["team"]
           if r["waves_per_simd"] < 3]
    assert not bad, json.dumps(bad[:10])


def test_no_scratch_except_the_x87_team_fold(kernels):
    bad = []
    for o, rows in kernels.items():
        for r in rows:
            allowed = 64 if "x87::ld_team_kernel<0" in r["kernel"] and (
                ", 7, " in r["kernel"] or ", 8, " in r["kernel"]) else 0
            if r["scratch"] > allowed:
                bad.append((o, r["kernel"][:100], r["scratch"], r["vgpr_spill"]))
    assert not bad, json.dumps(bad[:10])
