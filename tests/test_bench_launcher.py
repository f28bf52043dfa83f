"""bench.py's multi-rank launcher on the CPU (gloo, --dry-run: no HIP call).

The driver runs `bench.py --gpus N` both bare and under torch.distributed.run; either way the JSON line
must describe N ranks, and a launcher whose WORLD_SIZE disagrees with --gpus must be refused rather
than measured (the reference's multi-process use is scripts/train_dnerf.sh:3-12)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_bare_bench_spawns_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    j = _json_line(r.stdout)
    assert j["n_gpus"] == 2 and j["dry_run"] is True
    assert [p["rank"] for p in j["per_rank"]] == [0, 1]
    # each rank's own step result reached rank 0 (num_rendered stand-in = 1000 + rank)
    assert [p["num_rendered"] for p in j["per_rank"]] == [1000, 1001]
    assert j["ms_per_step"] == max(p["ms_per_step"] for p in j["per_rank"])


def test_driver_style_launch():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), BENCH, "--gpus", "2",
                        "--dry-run", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    j = _json_line(r.stdout)
    assert j["n_gpus"] == 2 and len(j["per_rank"]) == 2


def test_world_size_mismatch_is_refused():
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--dry-run"], capture_output=True, text=True,
                       timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0
    assert "refusing" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
