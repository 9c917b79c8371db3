"""C-ABI boundary checks that need no GPU.

* libosgpu_reduce.so loads and exports every function include/osgpu_reduce.h
  declares: the 44 shmem_<T>_<op>_to_all of the reference API
  (include/shmem/api.h:2173-2409, src/reductions.c:248-297), their pshmem_
  profiling names (include/pshmem.h:745-935), and the control surface.
* Host-side logic: fold order (src/reductions.c:84-111), shard ranges,
  the nreduce <= 0 collective (two barriers, src/reductions.c:82,113).
* The product fails loudly without a GPU instead of computing on the CPU.
"""
import ctypes
import os
import subprocess
import sys

import pytest

import osgpu
from support import team as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(osgpu.LIB_PATH):
        osgpu.build()
    return osgpu.load()


def test_exports_every_declared_symbol(lib):
    names = osgpu.header_symbols()
    assert len([n for n in names if n.endswith("_to_all")]) == 88
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", osgpu.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    kinds = {}
    for line in out.splitlines():
        parts = line.split()
        if len(parts) == 3:
            kinds[parts[2]] = parts[1]
    for e in osgpu.ENTRY_POINTS:
        assert kinds.get("p" + e) == "T", e         # pshmem_*: strong
        assert kinds.get(e) in ("W", "V"), e        # shmem_*: weak alias


def test_header_compiles_as_c_and_cxx(tmp_path):
    src = tmp_path / "use.c"
    src.write_text('#include "osgpu_reduce.h"\n'
                   'int main(void){ void (*f)(double*,double*,int,int,int,int,double*,long*)'
                   ' = shmem_double_sum_to_all; return f == 0; }\n')
    inc = os.path.join(ROOT, "include")
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-c", str(src), "-I", inc,
                    "-o", str(tmp_path / "a.o")], check=True)
    cpp = tmp_path / "use.cpp"
    cpp.write_text('#include "osgpu_reduce.h"\n'
                   'int main(){ auto f = &shmem_complexd_prod_to_all; return f == nullptr; }\n')
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-c", str(cpp), "-I", inc,
                    "-o", str(tmp_path / "b.o")], check=True)


def test_link_a_c_program_against_the_library(tmp_path):
    """A C application links the drop-in exactly like the reference's
    libshmem (no GPU call happens: nreduce = 0 only synchronises)."""
    src = tmp_path / "app.c"
    src.write_text(r'''
#include <stdio.h>
#include "osgpu_reduce.h"
static int me(void){ return 0; }
static int np(void){ return 1; }
static int nbar = 0;
static void bar(int a, int b, int c, long *p){ (void)a;(void)b;(void)c;(void)p; nbar++; }
int main(void){
  osgpu_pe_ops ops = { me, np, bar, 0 };
  if (osgpu_set_pe_ops(&ops)) return 2;
  long psync[OSGPU_REDUCE_SYNC_SIZE] = {0};
  double t[1], s[1], w[OSGPU_REDUCE_MIN_WRKDATA_SIZE];
  shmem_double_sum_to_all(t, s, 0, 0, 0, 1, w, psync);
  pshmem_int_max_to_all((int*)t, (int*)s, 0, 0, 0, 1, (int*)w, psync);
  printf("%d\n", nbar);
  return nbar == 4 ? 0 : 1;
}
''')
    exe = tmp_path / "app"
    subprocess.run(["gcc", "-std=c11", str(src), "-I", os.path.join(ROOT, "include"),
                    "-L", os.path.dirname(osgpu.LIB_PATH), "-losgpu_reduce",
                    "-Wl,-rpath," + os.path.dirname(osgpu.LIB_PATH), "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "4"


def test_single_hip_runtime_in_process():
    """Loading the library and torch in either order maps exactly one
    libamdhip64 (two runtimes in one process corrupt the heap at exit)."""
    code = (
        "import sys; sys.path[:0]=[%r]\n"
        "import osgpu; osgpu.load()\n"
        "import torch\n"
        "maps = open('/proc/self/maps').read().split('\\n')\n"
        "print(len({l.split()[-1] for l in maps if 'libamdhip64' in l}))\n"
    ) % os.path.join(ROOT, "test-resilient-osss-ucx_amd")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip() == "1"


def test_has_op_matches_reference_table(lib):
    import oracle as O
    for ti, t in enumerate(O.TYPES):
        for oi, o in enumerate(O.OPS):
            assert lib.osgpu_has_op(ti, oi) == int(O.has_op(t, o))
    sizes = [2, 4, 8, 8, 4, 8, 16, 8, 16]
    assert [lib.osgpu_type_size(i) for i in range(9)] == sizes


def test_fold_order_matches_reference_walk(lib):
    import oracle as O
    for (ps, ls, sz) in ((0, 0, 1), (0, 0, 8), (1, 1, 3), (2, 0, 4), (0, 2, 2), (3, 0, 5)):
        for me in O.active_set(ps, ls, sz):
            assert osgpu.fold_order(me, ps, ls, sz) == O.fold_order(me, ps, ls, sz)
    with pytest.raises(ValueError):
        osgpu.fold_order(1, 0, 1, 2)   # PE 1 is not in {0, 2}


@pytest.mark.parametrize("eb", [2, 4, 8, 16])
def test_shard_ranges_partition(lib, eb):
    for n in (0, 1, 7, 63, 64, 65, 1000, 4097, 1 << 20, (1 << 20) + 3):
        for P in (1, 2, 3, 4, 7, 8):
            prev = 0
            for i in range(P):
                lo, hi = osgpu.shard_range(n, P, i, eb)
                assert lo == prev and hi >= lo
                if i < P - 1:
                    assert (lo * eb) % 16 == 0 and (hi * eb) % 16 == 0
                prev = hi
            assert prev == n


def test_zero_length_collective_only_synchronises(lib):
    tm = T.Team(4, 4096, device=False)
    for t, op in (("int", "sum"), ("double", "max"), ("complexd", "prod")):
        before = [tm.pet.pet_barrier_calls(pe) for pe in range(4)]
        tm.run(t, op, 1024, 0, 0)
        after = [tm.pet.pet_barrier_calls(pe) for pe in range(4)]
        assert [a - b for a, b in zip(after, before)] == [2, 2, 2, 2]


@pytest.mark.parametrize("call", ["tm.run('int', 'sum', 1024, 0, 8)",
                                  "tm.run_coll('fcollect', 32, 1024, 0, 8)"])
def test_fails_loudly_without_gpu(call):
    """Host-memory call on a machine with no GPU (a reduction, and a
    data-movement collective): abort with a message, never a CPU result."""
    code = (
        "import sys, ctypes; sys.path[:0]=[%r, %r, %r]\n"
        "import numpy as np\n"
        "from support import team as T\n"
        "tm = T.Team(2, 4096, device=False)\n"
        "tm.write(0, 0, np.arange(8, dtype=np.int32)); tm.write(1, 0, np.arange(8, dtype=np.int32))\n"
        "%s\n"
        "print('COMPUTED')\n"
    ) % (os.path.join(ROOT, "tests"), os.path.join(ROOT, "test-resilient-osss-ucx_amd"),
         os.path.join(ROOT, "oracle"), call)
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode != 0
    assert "COMPUTED" not in r.stdout
    assert "osgpu_reduce" in r.stderr


def test_missing_runtime_is_reported():
    code = (
        "import sys, ctypes; sys.path[:0]=[%r]\n"
        "import osgpu\n"
        "L = osgpu.load(); L.osgpu_set_pe_ops(None)\n"
        "buf = (ctypes.c_int*8)()\n"
        "L.shmem_int_sum_to_all(buf, buf, 8, 0, 0, 1, buf, (ctypes.c_long*128)())\n"
    ) % os.path.join(ROOT, "test-resilient-osss-ucx_amd")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode != 0
    assert "no OpenSHMEM runtime" in r.stderr
