"""The CPU restatement (oracle/) against the reference's golden vectors.

Element ops: tests/golden/ops_<type>.npz hold the outputs of the reference's
own src/shmemu/miscops.c (compiled unmodified, oracle/_ref).  Reduce cases:
tests/golden/reduce_cases.json hold SHA-256 digests of per-PE targets folded
with those reference ops in the order of src/reductions.c:79-111.
"""
import os

import numpy as np
import pytest

import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("t", O.TYPES)
def test_element_ops_match_reference(t):
    z = np.load(os.path.join(GOLD, f"ops_{t}.npz"))
    a = O.from_value_bytes(t, z["a"])
    b = O.from_value_bytes(t, z["b"])
    nops = 0
    for op in O.OPS:
        if not O.has_op(t, op):
            assert "out_" + op not in z
            continue
        got = O.value_bytes(O.op_elementwise(t, op, a, b))
        want = z["out_" + op]
        bad = np.nonzero((got.reshape(a.size, -1) != want.reshape(a.size, -1)).any(1))[0]
        assert bad.size == 0, f"{t}/{op}: {bad.size} mismatches, first at {bad[:5]}"
        nops += 1
    assert nops >= 2


def test_all_44_entry_points_exist():
    assert len(O.ALL_PAIRS) == 44
    assert sum(1 for t, o in O.ALL_PAIRS if o == "sum") == 9
    assert sum(1 for t, o in O.ALL_PAIRS if o in ("max", "min")) == 14


def test_fold_order():
    # src/reductions.c:84-111: me first, then ascending active set skipping me
    assert O.fold_order(2, 0, 0, 4) == [2, 0, 1, 3]
    assert O.fold_order(3, 1, 1, 3) == [3, 1, 5]
    assert O.fold_order(0, 0, 2, 2) == [0, 4]


CASES = O.load_cases()


def _chunks(n):
    return [CASES[i::n] for i in range(n)]


@pytest.mark.parametrize("chunk", range(8))
def test_reduce_cases_match_golden(chunk):
    for c in _chunks(8)[chunk]:
        src = O.case_inputs(c)
        out = O.to_all(c["type"], c["op"], src, c["PE_start"], c["logPE_stride"],
                       c["PE_size"])
        for pe, dg in c["digests"].items():
            got = O.digest(out[int(pe)])
            assert got == dg, (f"{c['type']}/{c['op']} P={c['npes']} N={c['nreduce']} "
                               f"{c['tag']} PE {pe}")
            if pe in c["hex"]:
                assert O.value_bytes(out[int(pe)]).tobytes().hex() == c["hex"][pe]


def test_fp_results_depend_on_pe():
    """each PE folds in its own order, so FP sums differ by PE."""
    c = next(c for c in CASES if c["tag"] == "order" and c["type"] == "double")
    assert len(set(c["digests"].values())) > 1
    c = next(c for c in CASES if c["tag"] == "config3")
    assert len(set(c["digests"].values())) == 1


def test_reference_lib_agrees_when_present():
    if O.ref_lib() is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    t, op = "complexd", "prod"
    a = O.gen_input(t, 5000, 1, "edge")
    b = O.gen_input(t, 5000, 2, "edge")
    assert np.array_equal(O.value_bytes(O.op_elementwise(t, op, a, b)),
                          O.value_bytes(O.op_elementwise(t, op, a, b, use_ref=True)))


def test_cpu_baseline_runs():
    src = O.team_inputs("double", 2, 4096, 7, "unit12")
    sec = O.cpu_baseline("double", "sum", src, reps=3, pin=False)
    assert 0 < sec < 1.0


@pytest.mark.parametrize("tpp", [1, 3, 8])
@pytest.mark.parametrize("t,op,P", [("double", "sum", 2), ("long", "xor", 3), ("float", "min", 4),
                                    ("int", "sum", 2)])
def test_cpu_baseline_results(t, op, P, tpp):
    # the timed baseline computes the reference's results: every PE's target
    # equals the oracle's fold in that PE's order, whatever the thread split
    # (ragged n: the parts and the 64-element chunks do not divide it)
    n = 64 * 37 + 5
    src = O.team_inputs(t, P, n, 11, "unit12" if t in ("double", "float") else "bits")
    got = []
    sec = O.cpu_baseline(t, op, src, reps=1, pin=False, threads_per_pe=tpp, targets=got)
    assert 0 < sec < 1.0
    want = O.to_all(t, op, src)
    for pe in range(P):
        assert np.array_equal(np.asarray(got[pe]).view(np.uint8),
                              np.asarray(want[pe]).view(np.uint8)), pe
    # the same loop calling the reference's own compiled element function
    # (oracle/_ref, src/shmemu/miscops.c) through the pointer, as
    # src/reductions.c:95-96 does -- the form bench.py's cpu_baseline times
    if O.ref_lib() is not None:
        got = []
        O.cpu_baseline(t, op, src, reps=1, pin=False, threads_per_pe=tpp, targets=got,
                       ref_ops=True)
        for pe in range(P):
            assert np.array_equal(np.asarray(got[pe]).view(np.uint8),
                                  np.asarray(want[pe]).view(np.uint8)), pe
