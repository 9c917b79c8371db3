"""The CPU restatement and the host build of the x87 soft-float under
AddressSanitizer + UndefinedBehaviorSanitizer ("Race detection
/ sanitizers": the reference has none; its debug argument checks are
compiled out).  Each build runs the CPU tests that exercise it, in a child
process with the sanitizer runtime preloaded (host code only; nothing here
touches a GPU):

* oracle/ (oracle_ops.c, oracle_reduce.c, oracle_coll.c) built by gcc with
  -fsanitize=address,undefined: tests/test_oracle.py (golden vectors, every
  (type, op), fold orders, in-place, active subsets, the CPU-baseline loop
  shapes with their threads) and tests/test_collectives.py;
* csrc/x87.hpp compiled for the host by hipcc with the same sanitizers
  (-Xarch_host, so no device code is instrumented): tests/test_x87_softfloat.py
  (2 M random encodings, the fast add's gap / carry / cancellation seams, the
  team folds at 2-8 members).

A planted out-of-range shift first proves the runtime aborts on undefined
behaviour, so a green run means none was executed.
"""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
SAN_HOST = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
            "-Xarch_host", "-fno-sanitize-recover=undefined", "-Xarch_host", "-shared-libsan"]
ENV = {"ASAN_OPTIONS": "detect_leaks=0", "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}


def _clang_asan():
    libs = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return libs[-1] if libs else None


def _gcc_asan():
    try:
        p = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True)
    except FileNotFoundError:
        return None
    path = p.stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


def _pytest(files, env_extra, preload):
    env = dict(os.environ, **ENV, **env_extra)
    env["LD_PRELOAD"] = preload
    return subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                           "-m", "not gpu"] + files, cwd=ROOT, env=env, capture_output=True,
                          text=True, timeout=900)


def test_sanitizer_runtime_catches_undefined_behaviour(tmp_path):
    rt = _clang_asan()
    if not rt or not os.path.exists(HIPCC):
        pytest.skip("no clang sanitizer runtime")
    src = tmp_path / "ub.hip"
    src.write_text('#include <stdint.h>\n'
                   'extern "C" uint64_t ubshift(uint64_t x, unsigned n) { return x << n; }\n')
    lib = tmp_path / "libub.so"
    subprocess.run([HIPCC, "-O1", "-g", "-fPIC", "-shared"] + SAN_HOST + [str(src), "-o", str(lib)],
                   check=True, capture_output=True)
    code = ("import ctypes; L = ctypes.CDLL(%r); L.ubshift.restype = ctypes.c_uint64;"
            "L.ubshift.argtypes = [ctypes.c_uint64, ctypes.c_uint];"
            "assert L.ubshift(1, 3) == 8; L.ubshift(1, 64)" % str(lib))
    p = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **ENV, LD_PRELOAD=rt),
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "shift exponent 64" in p.stderr, p.stderr[-2000:]


def test_oracle_under_asan_ubsan(tmp_path):
    rt = _gcc_asan()
    if not rt:
        pytest.skip("no gcc libasan")
    lib = tmp_path / "liboracle_san.so"
    od = os.path.join(ROOT, "oracle")
    subprocess.run(["gcc", "-O1", "-g", "-std=gnu11", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
                    "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=undefined", "-shared", "-o", str(lib)] +
                   [os.path.join(od, f) for f in ("oracle_ops.c", "oracle_reduce.c", "oracle_coll.c")] +
                   ["-lpthread", "-lm"], check=True, capture_output=True)
    p = _pytest(["tests/test_oracle.py", "tests/test_collectives.py"], {"ORACLE_LIB": str(lib)}, rt)
    assert p.returncode == 0, (p.stdout + p.stderr)[-4000:]
    assert "passed" in p.stdout and "runtime error" not in p.stderr


def test_x87_host_build_under_asan_ubsan(tmp_path):
    rt = _clang_asan()
    if not rt or not os.path.exists(HIPCC):
        pytest.skip("no clang sanitizer runtime")
    lib = tmp_path / "libx87check_san.so"
    subprocess.run([HIPCC, "-O1", "-g", "-fPIC", "-shared", "-std=c++17"] + SAN_HOST +
                   [os.path.join(ROOT, "tests", "support", "x87_check.hip"), "-o", str(lib)],
                   check=True, capture_output=True)
    p = _pytest(["tests/test_x87_softfloat.py"], {"X87CHECK_LIB": str(lib)}, rt)
    assert p.returncode == 0, (p.stdout + p.stderr)[-4000:]
    assert "passed" in p.stdout and "runtime error" not in p.stderr
