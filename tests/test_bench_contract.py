"""bench.py's host-side contract pieces, on CPU: the roofline object (achieved = algorithmic
bytes per launch / average launch time; traffic from the committed rocprofv3 PMC summary of
the same per-launch workload; the access pattern's measured ceiling beside the spec peak)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_roofline_headline_workload():
    b = load_bench()
    per = 8192 << 20  # BASELINE config 2: 8192 x 1 MiB per launch
    r = b.roofline((10 * 1.25, 10, 10 * per), b.HBM_PEAK_GBPS)  # 10 launches of 1.25 ms
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["achieved"] - per / 1.25e-3 / 1e9) < 0.1
    assert abs(r["frac"] - r["achieved"] / 8000.0) < 1e-4
    assert r["algorithmic_bytes_per_launch"] == per
    # the committed PMC summary of this workload supplies HBM traffic, within 0.1 % of it
    assert r["traffic"] is not None and abs(r["traffic"] / per - 1) < 1e-3
    assert os.path.exists(os.path.join(ROOT, r["traffic_source"]))
    assert r["pattern_ceiling"]["achieved"] < 8000.0


def test_roofline_update_workload_and_unmatched_sizes():
    b = load_bench()
    per = 3 * 4096 * 100000  # BASELINE config 3: new + old + write-back per 4 KiB block write
    r = b.roofline((0.25, 1, per), b.HBM_PEAK_GBPS, kernel="upd_delta_kernel")
    assert r["kernel"] == "upd_delta_kernel" and r["traffic"] is not None
    assert abs(r["traffic"] / per - 1) < 1e-2
    # no PMC summary for another per-launch size: traffic stays null rather than borrowed
    r = b.roofline((1.0, 1, per + 4096), b.HBM_PEAK_GBPS, kernel="upd_delta_kernel")
    assert r["traffic"] is None
