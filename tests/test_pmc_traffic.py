"""tools/pmc_traffic.traffic(): the HBM-bytes arithmetic behind the bench
line's roofline.traffic (live passes and profiles/ files alike), on
synthetic rocprofv3 counter CSVs -- no GPU."""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import pmc_traffic  # noqa: E402

FIELDS = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"]


def _write(d, counter, rows):
    os.makedirs(os.path.join(d, "host", "1234"), exist_ok=True)
    with open(os.path.join(d, "host", "1234", "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=FIELDS)
        w.writeheader()
        for i, (k, v) in enumerate(rows):
            w.writerow({"Dispatch_Id": i, "Kernel_Name": k, "Counter_Name": counter,
                        "Counter_Value": v})


def test_traffic_doubles_fetch_and_takes_medians(tmp_path):
    n = 1 << 20
    team = "void osgpu::team_vec_kernel<double, 0, 2, true>(osgpu::TeamPtrs<double, 2>, ...)"
    comb = "void osgpu::combine_vec_kernel<double, 0, 2>(...)"
    # the team kernel reads 2*n*8 and writes 2*n*8: FETCH_SIZE counts half (KiB)
    half_read_kib = 2 * n * 8 / 2 / 1024
    write_kib = 2 * n * 8 / 1024
    f, w = str(tmp_path / "f"), str(tmp_path / "w")
    _write(f, "FETCH_SIZE", [(team, half_read_kib), (team, half_read_kib + 4), (team, 1.0),
                             (comb, 123.0)])
    _write(w, "WRITE_SIZE", [(team, write_kib), (team, write_kib), (comb, 7.0)])
    r = pmc_traffic.traffic(f, w, n, "team_vec_kernel<double, 0, 2, true>", 32)
    assert r["launches"] == [3, 2]
    assert r["read_bytes"] == 2 * n * 8
    assert r["write_bytes"] == 2 * n * 8
    assert r["traffic_over_algorithmic"] == 1.0
    assert pmc_traffic.traffic(f, w, n, "team_lds_kernel<double, 0, 4, true, 4", 64) is None


def test_bench_labels_looked_up_traffic():
    sys.path.insert(0, ROOT)
    import bench
    bench.LIVE_TRAFFIC.clear()
    tr = bench.load_traffic(n=64 << 20)
    assert tr is not None and tr["source"].startswith("looked up: profiles/")
    bench.LIVE_TRAFFIC[bench.COMBINE_KERNEL] = {"nreduce": 64 << 20,
                                                              "source": "live", "bytes_per_launch": 1}
    try:
        assert bench.load_traffic(n=64 << 20)["source"] == "live"
        assert bench.load_traffic(n=32 << 20) is None or \
            bench.load_traffic(n=32 << 20)["source"] != "live"
    finally:
        bench.LIVE_TRAFFIC.clear()
