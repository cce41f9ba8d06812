"""bench.py's multi-rank launch contract on CPU (gloo): `--gpus N` outside torchrun starts
N ranks itself, the world size must equal --gpus, and the gathered outputs come back in
rank order (the stub step writes each rank's id into its out_flat slice)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    e["OMP_NUM_THREADS"] = "1"
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=REPO)


def _json_line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_gpus2_spawns_two_ranks_and_gathers_in_rank_order():
    r = _run(["--gpus", "2", "--cpu-dry-run", "--steps", "3", "--warmup", "1", "--batch", "2"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json_line(r.stdout)
    assert out["n_gpus"] == 2
    assert out["gather_check"] == "ok"


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "2", "--cpu-dry-run", "--steps", "1", "--warmup", "0"],
             env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "!= --gpus 2" in (r.stderr + r.stdout)


@pytest.mark.gpu
def test_gpus2_shared_gpu_rehearsal_runs_real_kernels():
    """The N-rank bench path on a one-GPU box: `--gpus 2` spawns two ranks that each plan,
    capture and replay the real HIP forward on cuda:0, time between barriers, take the max
    over ranks and all-gather out_flat (gloo, host-staged: RCCL refuses two ranks on one GPU).
    Rank 0's slice of the gathered buffer must be its own output."""
    r = _run(["--gpus", "2", "--shared-gpu-rehearsal", "--size", "n", "--batch", "4", "--steps", "3", "--warmup", "1",
              "--no-cpu-baseline", "--no-latency", "--no-secondary"], timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json_line(r.stdout)
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 8
    assert out["outputs_finite"] and out["gather_rank0_matches"]
    assert "rehearsal" in out and out["value"] > 0
