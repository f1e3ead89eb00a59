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


def test_roofline_config3_fused_kernels_carry_rocprof_and_the_phases_bound():
    """Round 5: the fused config-3 kernels (plain write-back stores) carry the committed profile's rocprof
    duration beside their own stamps, and the pattern ceiling is the phases bound (198.8 us per 100k writes)."""
    b = load_bench()
    per = 3 * 4096 * 100000
    for kern in ("upd_fused_kernel", "uio_afused_kernel"):
        r = b.roofline((0.225, 1, per), b.HBM_PEAK_GBPS, kernel=kern)
        assert r["traffic"] is not None and abs(r["traffic"] / per - 1) < 0.05, (kern, r)
        assert r["rocprof_avg_us"] > 0 and abs(r["frac_rocprof"] - per / (r["rocprof_avg_us"] * 1e-6) / 1e9 / 8000.0) < 1e-3
        assert "timing_note" in r
        assert abs(r["pattern_ceiling"]["achieved"] - per / 198.8e-6 / 1e9) < 2.0
        assert os.path.exists(os.path.join(ROOT, r["pattern_ceiling"]["source"]))


def _bench(args, env_extra=None, timeout=120):
    import json
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                       text=True, timeout=timeout)
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    return p.returncode, lines, p.stderr


def test_gpus_n_spawns_n_ranks_without_a_launcher():
    """`bench.py --gpus N` with WORLD_SIZE unset starts N ranks itself (RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* as torchrun sets them); rank 0 prints the one line."""
    rc, lines, err = _bench(["--gpus", "3", "--dry-run-launch", "-1"])
    assert rc == 0, err
    assert len(lines) == 1
    assert lines[0]["n_gpus"] == 3 and lines[0]["local_ranks"] == [0, 1, 2] and lines[0]["launched"]


def test_gpus_one_runs_in_process():
    rc, lines, err = _bench(["--gpus", "1", "--dry-run-launch", "-1"])
    assert rc == 0, err
    assert lines == [{"dry_run": True, "n_gpus": 1, "local_ranks": [0], "launched": False}]


def test_world_size_mismatch_fails():
    rc, lines, err = _bench(["--gpus", "2", "--dry-run-launch", "-1"], {"WORLD_SIZE": "4", "RANK": "0"})
    assert rc != 0 and not lines and "disagrees" in err


def test_failed_rank_fails_the_launch():
    """A rank that dies makes the launcher exit non-zero (the worst code) after a grace period
    that ends the ranks left waiting in the rendezvous."""
    rc, lines, err = _bench(["--gpus", "2", "--dry-run-launch", "1"], {"H3C_BENCH_GRACE_S": "3"})
    assert rc == 3 and not lines


def test_more_ranks_than_gpus_is_refused_unless_rehearsal():
    """WORLD_SIZE > visible GPUs exits non-zero; --allow-shared-devices allows it and
    the line then reports the distinct devices used (with "rehearsal": true)."""
    b = load_bench()
    assert b.check_devices(8, 8, False) is None and b.check_devices(1, 1, False) is None
    err = b.check_devices(8, 1, False)
    assert err and "allow-shared-devices" in err
    assert b.check_devices(8, 1, True) is None
    assert b.check_devices(2, 0, False)  # no GPU at all
    assert b.devices_used(8, 1) == 1 and b.devices_used(8, 8) == 8 and b.devices_used(2, 4) == 2


def test_oversubscribed_launch_exits_nonzero_on_cpu():
    """On this GPU-less container every real (non dry-run) rank sees 0 devices: the N=2 launch fails
    before any GPU work, with the reason on stderr."""
    rc, lines, err = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0"], {"H3C_BENCH_GRACE_S": "3"},
                            timeout=300)
    assert rc == 2 and not lines and "allow-shared-devices" in err
