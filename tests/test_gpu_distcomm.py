"""Two processes (torch.distributed.run children of this test, both on the box's one GPU, gloo process group)
drive MapAnything.enable_view_sharding() through the real DistComm: the asynchronous all-gather handle of the
overlapped global layers, the rank-0 scale-token broadcast and the rank-0 output gather (tests/dist_worker.py).
RCCL itself refuses two ranks on one device, so the group is gloo here; the code path above the collective calls is
the production one."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_errors(r):
    """The ranks' own tracebacks ([rankN]: lines), which torch.distributed.run's summary would push out of view."""
    lines = [ln for ln in (r.stdout + r.stderr).splitlines() if ln.startswith("[rank")]
    return "\n".join(lines[-80:]) or (r.stdout[-3000:] + r.stderr[-3000:])


def test_two_process_view_sharding_over_distcomm(tmp_path):
    prefix = str(tmp_path / "res")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(HERE, "dist_worker.py"), prefix]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, _rank_errors(r)
    res = [json.load(open(f"{prefix}.{k}.json")) for k in range(2)]
    for ov in ("1", "0"):
        s = res[0][f"scales_{ov}"]
        assert s[0] == s[1], s  # one metric scale on every rank (rank 0's scale token)
        assert res[0][f"n_views_{ov}"] == 3 and res[1][f"n_views_{ov}"] == 1  # gathered on rank 0 only
        err = res[0][f"err_{ov}"]
        assert all(e < 2e-5 for e in err.values()), (ov, err)


def test_one_rank_rccl_sharded_graph(tmp_path):
    """A real one-rank RCCL process group (tests/nccl1_worker.py, MAPA_FORCE_COLLECTIVES=1): the sharded forward with
    its K/V all-gathers and scale-token broadcast through RCCL (the direct, non-blocking-initialised communicator),
    eager and HIP-graph captured / replayed, in fp32 and in the bf16 recipe — in the gather-first form and, with
    MAPA_FORCE_OVERLAP=1, in the overlapped form every N > 1 global layer takes (side-stream all-gather forked and
    joined inside the capture, local / remote attention, LSE merge).  Graph-replayed == eager bitwise; sharded ==
    unsharded (fp32 within 2e-5: the sharded global layers project Q and K/V in two GEMMs, attend through the segment
    table, and in the overlapped form merge two partials).  Mode "scenes2": two batched scenes per view through the
    batched-scene sharded layers (ShardPlan.scenes = 2), against the unsharded batched forward; mode "geoscenes2":
    two batched scenes with mixed geometric inputs (b2_224), the per-scene camera normalisation and per-image camera
    picking captured on the shard — in the bf16 recipe with the default TF32-equivalent heads too."""
    out = str(tmp_path / "nccl1.json")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(HERE, "nccl1_worker.py"), out]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, _rank_errors(r)
    res = json.load(open(out))
    print("\n[one-rank RCCL sharded forward]", json.dumps(res, indent=1))
    for mode in ("gather", "overlap", "scenes2", "geoscenes2"):
        for prec in ("fp32", "bf16"):
            d = res[f"{mode}_{prec}"]
            assert d["direct_rccl"] and d["sharded_graph_keys"] == 1, d
            assert d["graph_eq_eager"] and d["replay_eq_eager"], d
            assert d["replay_python_merges"] == 0, d  # the replay launches nothing from Python
            assert d["eager_merges"] == (12 if mode == "overlap" else 0), d  # one merge per global layer
        assert all(e < 2e-5 for e in res[f"{mode}_fp32"]["err_vs_single"].values()), res[f"{mode}_fp32"]


def test_library_comm_c_abi_one_rank():
    """include/mapa.h mapa_comm_*: the library's own RCCL communicator (what a non-Python host of libmapa.so drives
    the sharded forward with), one rank: non-blocking init polled to ready, the K/V slot all-gather and the scale-token
    broadcast enqueued on the stream (identity at one rank), also captured into a HIP graph and replayed, the async
    error check, finalize / destroy; a second communicator is aborted instead."""
    import torch

    from mapanything import _native as nat

    uid = nat.CComm.unique_id()
    assert len(uid) == nat.lib().mapa_comm_unique_id_bytes() == 128
    c = nat.CComm(1, 0, uid, torch.cuda.current_device(), timeout_s=120)
    full = torch.randn(1000, 1536, device="cuda").to(torch.bfloat16)
    keep = full.clone()
    c.allgather_slots(full, 1000)
    tok = torch.randn(768, device="cuda")
    tk = tok.clone()
    c.broadcast_(tok, 0)
    torch.cuda.synchronize()
    assert torch.equal(full, keep) and torch.equal(tok, tk)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        full.mul_(2)
        c.allgather_slots(full, 1000)
        c.broadcast_(tok, 0)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(full, keep * 2) and torch.equal(tok, tk)
    c.check_async()
    del g
    c.close()
    c2 = nat.CComm(1, 0, nat.CComm.unique_id(), torch.cuda.current_device(), timeout_s=120)
    c2.close(abort=True)
    with pytest.raises(nat.NativeError):
        nat.CComm(2, 5, uid, torch.cuda.current_device())  # rank out of range: refused before any RCCL call
