"""bench.py's multi-rank harness on CPU: `--gpus N` without a launcher starts N
ranks itself; --cpu-stub runs the transmit bench's rank / RCCL-broadcast (here gloo) / barrier /
max-over-ranks code with a CPU stub pipeline.  The nccl path differs only in the backend and the
pipeline object."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=ROOT)


def test_bench_spawns_ranks_gloo_stub():
    r = _bench("--gpus", "2", "--cpu-stub", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--batch", "64")
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1                       # only rank 0 prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["global_batch"] == 128
    assert out["config"]["parallelism"] == "subframe-sharded x2"
    assert out["config"]["G"] == [86400, 86400]  # parameter block broadcast from rank 0 intact
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert len(out["per_rank_subframes_per_s"]) == 2 and min(out["per_rank_subframes_per_s"]) > 0
    assert 0 < out["rank_efficiency"] <= 1.0 + 1e-9


def test_bench_failing_rank_fails_the_job():
    r = _bench("--gpus", "2", "--cpu-stub", "--config", "C5", "--steps", "1", "--warmup", "0")
    assert r.returncode != 0


def test_bench_world_mismatch_rejected():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cpu-stub"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode == 2


def test_cpu_baseline_fields():
    sys.path.insert(0, ROOT)
    import bench
    cb = bench.cpu_baseline("C1", 0.5, 7)
    assert cb["cores"] == 1 and cb["value"] > 0
    assert cb["cores_all"] >= 1 and cb["value_all_cores"] > 0 and cb["cpu_model"]
    assert set(cb["stage_us_per_subframe"]) == set(cb["stage_impl"])
    # with the reference tree built here, the stages that have a buildable TU run the reference
    if os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libref_rm.so")):
        assert cb["kind"] == "reference+port"
        assert cb["stage_impl"]["rate_matching"] == "reference" and cb["stage_impl"]["ofdm_mod"] == "reference"
        assert cb["stage_impl"]["segmentation"] == "reference"
        if os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libref_mod.so")):
            # dlsch_modulation.c / dlsch_scrambling.c: only the turbo encoder stays a port
            assert cb["stage_impl"]["modulation"] == "reference" and cb["stage_impl"]["scrambling"] == "reference"
            assert cb["stage_impl"]["turbo_encoder"] == "port" and cb["port_share"] < 0.5
        assert 0 < cb["port_share"] < 1
