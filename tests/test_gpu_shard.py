"""Trace-sharded PageRank on the GPU: two processes share one GPU, each holding half
of a window's traces; collectives go through the host-staged backend over gloo.  The weights
must equal the whole graph's on one GPU (the per-iteration P_sr r sums are exact integers, so
only the once-per-graph preference sums may round differently), coverage exactly, and both
ranks bitwise.  A one-rank RCCL communicator exercises the RCCL plumbing of the same path."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from test_dist_gloo import _shard, _window_graph

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _whole(anomaly):
    from gpu_util import host_graph_from_oracle
    from microrank_amd import _lib
    from microrank_amd.graph import DeviceGraph

    ctx = _lib.Context(0)
    dg = DeviceGraph.upload(ctx, host_graph_from_oracle(_window_graph()))
    dg.pagerank(anomaly)
    w, cov = dg.fetch()
    dg.close()
    ctx.close()
    return w, cov


def _worker(rank, world, port, anomaly, backend, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gpu_util import host_graph_from_oracle
        from microrank_amd import _lib, shard
        from microrank_amd.graph import DeviceGraph

        ctx = _lib.Context(0)
        if backend == "host":
            shard.use_host(ctx)
        else:
            shard.use_rccl(ctx)
        dg = DeviceGraph.upload(ctx, host_graph_from_oracle(_shard(_window_graph(), rank, world)))
        w, cov = shard.sharded_pagerank(dg, anomaly)
        info = dg.info()
        dg.close()
        ctx.close()
        q.put((rank, w, cov, info))
    except Exception as e:   # surface the failure in the parent
        q.put((rank, repr(e), None, None))
    finally:
        dist.destroy_process_group()


def _run(world, anomaly, backend):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, anomaly, backend, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in res:
        assert r[2] is not None, f"rank {r[0]} failed: {r[1]}"
    return sorted(res, key=lambda r: r[0])


@pytest.mark.parametrize("anomaly", [False, True])
def test_two_shards_one_gpu_match_whole_graph(anomaly):
    w_ref, cov_ref = _whole(anomaly)
    res = _run(2, anomaly, "host")
    for rank, w, cov, info in res:
        np.testing.assert_allclose(w, w_ref, rtol=1e-12, atol=0)
        np.testing.assert_array_equal(cov, cov_ref)
    assert res[0][1].tobytes() == res[1][1].tobytes(), "ranks disagree"
    assert res[0][3]["T"] + res[1][3]["T"] == _window_graph().T


def test_one_rank_rccl_matches_whole_graph():
    w_ref, cov_ref = _whole(True)
    (rank, w, cov, info), = _run(1, True, "rccl")
    np.testing.assert_allclose(w, w_ref, rtol=1e-12, atol=0)
    np.testing.assert_array_equal(cov, cov_ref)
