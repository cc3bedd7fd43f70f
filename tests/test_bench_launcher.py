"""Multi-rank control path on CPU (no GPU): `bench.py --gpus N` starts N ranks itself when no launcher did, the
rank count it measures is asserted, a failing rank makes the job exit non-zero, and a dead peer turns a DistComm
collective into CommError within MAPA_COMM_TIMEOUT_S instead of a hang (parallel.init_distributed / DistComm)."""

import json
import os
import socket
import subprocess
import sys

import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    env.update(extra)
    return env


def _bench(args, **env):
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO, env=_env(**env),
                          capture_output=True, text=True, timeout=180)


def test_bench_gpus_n_launches_n_ranks():
    r = _bench(["--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["world_size_observed"] == 2 and line["dry_run"]
    # the N > 1 line explains its own overlap: per-layer all-gather vs local / remote attention (bench.kv_overlap)
    kvo = line["kv_overlap"]
    for k in ("allgather_ms_per_layer", "local_attn_ms", "remote_attn_ms", "gather_wait_ms", "overlap_frac"):
        assert k in kvo and kvo[k] is not None and kvo[k] >= 0, (k, kvo)


def test_bench_stdout_is_one_json_line_despite_native_prints():
    """Native libraries print to fd 1 (RCCL's version banner at communicator init, on every N > 1 rank): bench.py sends
    fd 1 to stderr and writes rank 0's JSON line to a private dup of the real stdout, so the job's stdout is exactly
    that one line (the driver parses it)."""
    r = _bench(["--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1"], MAPA_BENCH_STDOUT_NOISE="1")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    assert json.loads(lines[0])["dry_run"]
    assert "native stdout noise" in r.stderr


def test_bench_failing_rank_fails_the_job():
    r = _bench(["--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1", "--fail-rank", "1"])
    assert r.returncode != 0
    assert "injected failure" in r.stderr


def test_bench_rejects_rank_count_mismatch():
    r = _bench(["--gpus", "2", "--dry-run"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0 and "--gpus 2 but WORLD_SIZE=1" in r.stderr


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _dead_peer_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      MAPA_COMM_TIMEOUT_S="20")
    sys.path.insert(0, os.path.join(REPO, "map-anything_amd"))
    from mapanything.parallel import CommError, DistComm, init_distributed

    r, w = init_distributed("gloo")
    assert (r, w) == (rank, world)
    comm = DistComm()
    if rank == 1:
        os._exit(0)  # the peer dies after init, before the first K/V exchange
    full = torch.zeros(world * 4, 8)
    try:
        comm.allgather_slots(full, 4)
        q.put("no error")
    except CommError as e:
        q.put(f"CommError: {e}")


def test_dead_peer_raises_comm_error_instead_of_hanging():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dead_peer_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    msg = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert msg.startswith("CommError: K/V all-gather failed on rank 0 of 2"), msg
