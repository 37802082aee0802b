"""bench.py's launch contract at N > 1 (BASELINE configs[3]).

CPU: --gpus that disagrees with a launcher's WORLD_SIZE is refused before any
GPU work; the backend rule (RCCL only when every rank has a GPU of its own).
GPU (the one-GPU box): `bench.py --gpus 2` with no launcher spawns two ranks
itself, both drive the engine on the box's GPU, the logits all-gather runs
over gloo (ranks share the GPU), and rank 0 prints ONE JSON line whose
n_gpus / global_batch / value follow the contract: value = 2 * 256 * steps /
max-over-ranks wall time.  Anchor: the gathered logits of
/root/reference/CUDA/resnet18-kernel-lab/cpp/fp32/runtime/infer_e2e.cu:206-219.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "DLQ_DIST_BACKEND")}
    env.update(kw)
    return env


def test_gpus_must_match_launcher_world_size():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--steps", "1", "--warmup", "0"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode != 0
    assert "--gpus 4 but WORLD_SIZE=2" in r.stderr
    assert '{"metric"' not in r.stdout


def test_backend_rule():
    sys.path.insert(0, ROOT)
    import bench
    old = os.environ.pop("DLQ_DIST_BACKEND", None)
    try:
        assert bench.dist_backend(8, 8) == "nccl"
        assert bench.dist_backend(2, 8) == "nccl"
        assert bench.dist_backend(2, 1) == "gloo"
        os.environ["DLQ_DIST_BACKEND"] = "gloo"
        assert bench.dist_backend(8, 8) == "gloo"
    finally:
        os.environ.pop("DLQ_DIST_BACKEND", None)
        if old is not None:
            os.environ["DLQ_DIST_BACKEND"] = old


@pytest.mark.gpu
def test_bench_gpus2_spawns_two_ranks(gpu):
    steps = 3
    cmd = [sys.executable, BENCH, "--gpus", "2", "--steps", str(steps), "--warmup", "1", "--prof-steps", "1",
           "--extras", "0", "--cpu-baseline-images", "0", "--oracle-images", "0"]
    r = subprocess.run(cmd, env=_env(DLQ_DIST_BACKEND="gloo"), capture_output=True, text=True, timeout=600,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["global_batch"] == 512 and out["config"]["per_gpu_batch"] == 256
    assert out["config"]["parallelism"] == "dp2"
    assert "gloo" in out["config"]["exchange"]
    assert out["steps"] == steps and out["scaling"] == "weak"
    # value = all ranks' images / max-over-ranks time; ms_per_step = that time / steps
    dt = out["ms_per_step"] * steps / 1e3
    assert out["value"] == pytest.approx(2 * 256 * steps / dt, rel=2e-3)
    assert "cpu_baseline" not in out  # rank 0 at N = 1 only
    # each spawned rank gets its share of the host's threads (bench.rank_env)
    sys.path.insert(0, ROOT)
    import bench
    assert out["config"]["host_threads_rank0"] == max(1, bench.host_threads() // 2)


def test_rank_env_splits_host_threads():
    sys.path.insert(0, ROOT)
    import bench
    env = bench.rank_env({"PATH": "/bin"}, 3, 8, 29500, 256)
    assert env["RANK"] == "3" and env["LOCAL_RANK"] == "3" and env["WORLD_SIZE"] == "8"
    assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29500"
    assert env["OMP_NUM_THREADS"] == "32" and env["PATH"] == "/bin"
    assert bench.rank_env({}, 0, 8, 1, 4)["OMP_NUM_THREADS"] == "1"


def test_spawn_ranks_kills_children_on_interrupt(tmp_path):
    """An interrupted parent leaves no rank behind (spawn_ranks' finally)."""
    script = tmp_path / "parent.py"
    script.write_text(
        "import sys, os, signal, threading\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import bench, subprocess\n"
        "bench.__file__ = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'child.py')\n"
        "def _term():\n"
        "    import time\n"
        "    d = os.path.dirname(os.path.abspath(__file__))\n"
        "    t0 = time.time()\n"
        "    ok = lambda f: os.path.exists(f) and os.path.getsize(f) > 0\n"
        "    while time.time() - t0 < 50 and not all(ok(os.path.join(d, 'pid%d' % r)) for r in (0, 1)):\n"
        "        time.sleep(0.05)\n"
        "    os.kill(os.getpid(), signal.SIGTERM)\n"
        "threading.Thread(target=_term, daemon=True).start()\n"
        "sys.exit(bench.spawn_ranks(2))\n")
    (tmp_path / "child.py").write_text(
        "import os, time\n"
        "open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'pid%s' % os.environ['RANK']), 'w')"
        ".write(str(os.getpid()))\n"
        "time.sleep(120)\n")
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 128 + 15, r.stderr[-2000:]
    for rank in (0, 1):
        assert (tmp_path / f"pid{rank}").exists(), f"rank {rank} never started (pid file missing)"
        pid = int((tmp_path / f"pid{rank}").read_text())
        alive = True
        try:
            os.kill(pid, 0)
        except ProcessLookupError:
            alive = False
        assert not alive, f"rank {rank} (pid {pid}) outlived the parent"
