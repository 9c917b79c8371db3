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


REF_INCLUDE = "/root/reference/include"


def _ref_pin_source(lang):
    """One translation unit holding the reference's own declarations
    (include/shmem.h -> shmem/api.h:2173-2409, the pshmem_ declarations of
    include/pshmem.h:745-935, COMPLEXIFY include/shmem/defs.h:14-19) and
    then ours: a signature that
    differs from the reference's is a conflicting declaration of the same
    extern "C" function, a compile error in C11 and in C++17.  Every one of
    the 88 reduce-to-all names (and the collectives both headers declare)
    is then taken as a pointer of the REFERENCE's declared type."""
    names = [n for n in osgpu.header_symbols()
             if n.endswith("_to_all") or any(k in n for k in ("broadcast", "collect", "alltoall"))]
    if lang == "c":
        body = "".join(f"  {{ __typeof__(&{n}) p = &{n}; sink((void (*)(void)) p); }}\n"
                       for n in names)
        pre = "static void sink(void (*p)(void)) { (void) p; }\n"
    else:
        body = "".join(f"  {{ decltype(&::{n}) p = &::{n}; sink(reinterpret_cast<void (*)()>(p)); }}\n"
                       for n in names)
        pre = "static void sink(void (*p)()) { (void) p; }\n"
    # include/pshmem.h does not compile on its own (int32 / int64 / uint32
    # at :695-699 are undeclared anywhere), so its declarations of the
    # reduce-to-all and fcollect names are read out of it at test time
    import re
    ptext = open(os.path.join(REF_INCLUDE, "pshmem.h")).read()
    pdecl = re.findall(r"void\s+pshmem_\w+(?:_to_all|broadcast\d+|collect\d+|alltoall\d+)\s*"
                       r"\([^;]*\);", ptext)
    assert len([d for d in pdecl if "_to_all" in d]) == 44
    psect = ('#ifdef __cplusplus\nextern "C" {\n#endif\n' + "\n".join(pdecl) +
             '\n#ifdef __cplusplus\n}\n#endif\n')
    return ('#include <shmem.h>\n' + psect + '#include "osgpu_reduce.h"\n' + pre +
            "int main(void) {\n" + body + "  return 0;\n}\n"), names


@pytest.mark.skipif(not os.path.isdir(REF_INCLUDE), reason="reference checkout absent")
@pytest.mark.parametrize("lang", ["c", "cxx"])
def test_header_matches_reference_header(tmp_path, lang):
    """include/osgpu_reduce.h against the reference's include/shmem.h and
    include/pshmem.h's declarations in one translation unit, -Wall -Werror; a planted
    signature change (nreduce int -> long in one entry point) fails it."""
    src, names = _ref_pin_source(lang)
    assert len([n for n in names if n.endswith("_to_all")]) == 88
    ext, cc, std = (".c", "gcc", "-std=c11") if lang == "c" else (".cpp", "g++", "-std=c++17")
    f = tmp_path / ("pin" + ext)
    f.write_text(src)

    def compile_with(inc):
        return subprocess.run([cc, std, "-Wall", "-Werror", "-c", str(f), "-I", REF_INCLUDE,
                               "-I", inc, "-o", str(tmp_path / "pin.o")],
                              capture_output=True, text=True)
    r = compile_with(os.path.join(ROOT, "include"))
    assert r.returncode == 0, r.stderr[-3000:]
    # planted: shmem_int_sum_to_all with a long nreduce
    planted = tmp_path / "planted"
    planted.mkdir()
    hdr = open(os.path.join(ROOT, "include", "osgpu_reduce.h")).read()
    marker = "OSGPU_DECL_ALL(shmem_)\n"
    assert marker in hdr
    hdr = hdr.replace(marker, marker + "void shmem_int_sum_to_all(int *target, int *source, long "
                      "nreduce, int PE_start, int logPE_stride, int PE_size, int *pWrk, "
                      "long *pSync);\n")
    (planted / "osgpu_reduce.h").write_text(hdr)
    r = compile_with(str(planted))
    assert r.returncode != 0
    assert "shmem_int_sum_to_all" in r.stderr


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


def test_copy_streams_come_from_different_queue_pools(lib):
    """The STAGED path's H2D and D2H streams take the lowest and the highest
    stream priority: HIP pools hardware queues per priority level, so the
    two directions never share a queue (sharing one, they took turns: 27.7
    GB/s each way instead of 44.5 -- the round-3 host-staged regression,
    profiles/r05_host_staged_streams.jsonl).  ROCm's range is (0, -1) on
    this image; a one-level range is refused (the library then gives each
    stream a CU-masked queue of its own)."""
    i, o = ctypes.c_int(7), ctypes.c_int(7)
    for least, greatest in ((0, -1), (1, -1), (0, -2)):
        assert lib.osgpu_copy_stream_priorities(least, greatest, ctypes.byref(i),
                                                ctypes.byref(o)) == 0
        assert (i.value, o.value) == (least, greatest) and i.value != o.value
    assert lib.osgpu_copy_stream_priorities(0, 0, ctypes.byref(i), ctypes.byref(o)) != 0
    assert lib.osgpu_copy_stream_priorities(0, -1, None, None) != 0


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


def test_test_hook_refused_in_production(lib, monkeypatch):
    """the preflight fault hook is not in the public header and
    is refused unless the process enables test hooks (OSGPU_TEST_HOOKS=1)."""
    monkeypatch.delenv("OSGPU_TEST_HOOKS", raising=False)
    hdr = open(os.path.join(ROOT, "include", "osgpu_reduce.h")).read()
    assert "osgpu_test_preflight_fault" not in hdr
    lib.osgpu_test_preflight_fault.argtypes = [ctypes.c_int, ctypes.c_int]
    assert lib.osgpu_test_preflight_fault(0, 1) != 0
    assert b"test hooks are off" in lib.osgpu_last_error()
    assert "osgpu_test_max_launch_threads" not in hdr
    lib.osgpu_test_max_launch_threads.argtypes = [ctypes.c_longlong]
    assert lib.osgpu_test_max_launch_threads(2048) != 0
    assert b"test hooks are off" in lib.osgpu_last_error()


def test_product_never_references_the_oracle():
    """nothing under the product (csrc/, osgpu/, the
    public header) includes, links, loads or calls oracle/ -- outside
    comments the word does not appear, and the built library has no
    dependency on liboracle / libref_ops."""
    import glob
    import re
    pkg = os.path.join(ROOT, "test-resilient-osss-ucx_amd")
    files = (glob.glob(os.path.join(pkg, "csrc", "*.hip")) + glob.glob(os.path.join(pkg, "csrc", "*.cpp"))
             + glob.glob(os.path.join(pkg, "csrc", "*.hpp")) + glob.glob(os.path.join(pkg, "csrc", "Makefile"))
             + glob.glob(os.path.join(pkg, "osgpu", "*.py"))
             + [os.path.join(ROOT, "include", "osgpu_reduce.h")])
    bad = []
    for f in files:
        src = open(f).read()
        if f.endswith(".py") or f.endswith("Makefile"):
            code = re.sub(r"#.*", "", src)
            code = re.sub(r'"""(.|\n)*?"""', "", code)
        else:
            code = re.sub(r"/\*(.|\n)*?\*/", "", src)
            code = re.sub(r"//.*", "", code)
        if re.search(r"oracle|ref_ops", code, re.IGNORECASE):
            bad.append(os.path.relpath(f, ROOT))
    assert not bad, bad
    so = os.path.join(pkg, "libosgpu_reduce.so")
    if os.path.exists(so):
        out = subprocess.run(["readelf", "-d", so], capture_output=True, text=True).stdout
        assert "oracle" not in out and "ref_ops" not in out
