"""Trace-sharded PageRank on the GPU: two processes share one GPU, each holding half
of a window's traces; collectives go through the host-staged backend over gloo.  The weights
must equal the whole graph's on one GPU (the per-iteration P_sr r sums are exact integers, so
only the once-per-graph preference sums may round differently), coverage exactly, and both
ranks bitwise.  A one-rank RCCL communicator exercises the RCCL plumbing of the same path.
The tile path (N > 16384, config C5; or forced with MR_NO_FUSED) sums fp64 per-op partials over
the ranks instead: equal to the whole graph within 1e-10, ranks bitwise."""
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


def _worker(rank, world, port, anomaly, backend, q, big=None, tile=False, walk_ranks=(), empty_last=False, peer=False,
            env=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.update(env or {})
    if tile is True or (tile and rank in tile):   # True: every rank; a tuple: those ranks
        os.environ["MR_NO_FUSED"] = "1"   # read once, at this process's first graph prepare
    if rank in walk_ranks:
        os.environ["MR_KIND_WALK"] = "1"   # kinds hashed by the per-thread int32 walk (read once)
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
        if peer:
            shard.use_peer(ctx)
        if big is None:
            g = _window_graph()
            bounds = [0] + [g.T] * world if empty_last else None   # rank 0 all traces, the rest none
            hg = host_graph_from_oracle(_shard(g, rank, world, bounds))
        else:
            from microrank_amd import synth
            hg = synth.big_graph(big[0], big[1], seed=3, shard=(rank, world))
        dg = DeviceGraph.upload(ctx, hg)
        w, cov = shard.sharded_pagerank(dg, anomaly, precision=big[2] if big else "fp64")
        info = dg.info()
        dg.close()
        ctx.close()
        q.put((rank, w, cov, info))
    except Exception as e:   # surface the failure in the parent
        q.put((rank, repr(e), None, None))
    finally:
        dist.destroy_process_group()


def _run(world, anomaly, backend, big=None, tile=False, walk_ranks=(), empty_last=False, peer=False, env=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, anomaly, backend, q, big, tile, walk_ranks,
                                               empty_last, peer, env))
             for r in range(world)]
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


@pytest.mark.parametrize("peer", [False, True])
@pytest.mark.parametrize("tile", [False, True])
def test_four_shards_one_gpu_match_whole_graph(tile, peer):
    """FOUR processes share the GPU, a quarter of the window's traces each: the r' maxima ride the
    all-reduce in four one-hot slots, the kind classes merge over four ranks.  peer: the
    per-iteration all-reduce goes through IPC-mapped receive regions (mr_comm_peer_enable: every
    rank writes its limbs into every rank's region and sums its own in rank order) instead of the
    host-staged collective.  Fused path: the whole graph's weights within 1e-12 (exact integer
    limbs); tile path (fp64 per-op sums): 1e-10; all ranks bitwise."""
    w_ref, cov_ref = _whole(True)
    res = _run(4, True, "host", tile=tile, peer=peer)
    for rank, w, cov, info in res:
        np.testing.assert_allclose(w, w_ref, rtol=1e-10 if tile else 1e-12, atol=0)
        np.testing.assert_array_equal(cov, cov_ref)
    for r in res[1:]:
        assert r[1].tobytes() == res[0][1].tobytes(), "ranks disagree"
    assert sum(r[3]["T"] for r in res) == _window_graph().T


@pytest.mark.parametrize("mode", ["fused-wait", "fused-spin", "split"])
def test_four_shards_peer_matches_host_collective_bitwise(mode):
    """The peer exchange and the host-staged all-reduce give bitwise the same weights on the fused
    path (both sum the same exact integer limbs).  fused-*: the exchange inside k_fx_b (mode-1
    blocks push their limbs and store their round flag, mode-2 blocks sum the R slots) -- with
    one waiting block before mode 2 (ranks sharing a device, the default here) or with every
    mode-2 block spinning on its own flags (the distinct-GPU form; safe here: the window graph's
    k_tr_a blocks are small); split: the separate push / reduce launches (MR_PEER_SPLIT)."""
    env = {"fused-wait": {}, "fused-spin": {"MR_PEER_SPIN": "1"}, "split": {"MR_PEER_SPLIT": "1"}}[mode]
    a = _run(4, False, "host", peer=False)
    b = _run(4, False, "host", peer=True, env=env)
    for x, y in zip(a, b):
        assert x[1].tobytes() == y[1].tobytes()
        np.testing.assert_array_equal(x[2], y[2])


def test_one_rank_rccl_matches_whole_graph():
    w_ref, cov_ref = _whole(True)
    (rank, w, cov, info), = _run(1, True, "rccl")
    np.testing.assert_allclose(w, w_ref, rtol=1e-12, atol=0)
    np.testing.assert_array_equal(cov, cov_ref)


def test_two_tile_path_shards_match_whole_graph():
    """Small window, both ranks forced onto the tile path: fp64 op-sum all-reduce."""
    w_ref, cov_ref = _whole(True)
    res = _run(2, True, "host", tile=True)
    for rank, w, cov, info in res:
        np.testing.assert_allclose(w, w_ref, rtol=1e-10, atol=0)
        np.testing.assert_array_equal(cov, cov_ref)
    assert res[0][1].tobytes() == res[1][1].tobytes(), "ranks disagree"


def _union_of_shards(n_ops, n_traces, world):
    """The whole graph the shards of synth.big_graph(shard=(r, world)) make up."""
    from microrank_amd import synth
    from microrank_amd.graph import HostGraph

    parts = [synth.big_graph(n_ops, n_traces, seed=3, shard=(r, world)) for r in range(world)]
    sr_ops = np.concatenate([p.sr_ops for p in parts])
    offs = [parts[0].sr_off]
    for p in parts[1:]:
        offs.append(offs[-1][-1] + p.sr_off[1:])
    T = sum(p.T for p in parts)
    return HostGraph(range(n_ops), range(T), np.concatenate(offs), sr_ops, None, None,
                     np.concatenate([p.len_t for p in parts]), sum(p.len_o for p in parts), parts[0].ss_off,
                     parts[0].ss_par, parts[0].nchild, None, None)


@pytest.mark.parametrize("n_ops,precision", [(20_000, "fp64"), (20_000, "fp32"), (10_000, "fp64")])
def test_large_op_count_shards_match_whole_graph(n_ops, precision):
    """C5-shaped (N = 20000 > the fused path's 16384: tile path), power-law ops, 2 ranks x 30k
    traces on one GPU vs the union graph on one GPU and vs the oracle.  N = 10000 (C4's op
    count): the fused path with ops relabelled by coverage -- each rank by its OWN shard's
    coverage, so the ranks' labels differ and the exchange must stay in the graph's op order."""
    from microrank_amd import _lib
    from microrank_amd.graph import DeviceGraph

    n_tr = 30_000
    hg = _union_of_shards(n_ops, n_tr, 2)
    ctx = _lib.Context(0)
    dg = DeviceGraph.upload(ctx, hg)
    dg.pagerank(True, precision=precision)
    w_ref, cov_ref = dg.fetch()
    dg.close()
    ctx.close()
    res = _run(2, True, "host", big=(n_ops, n_tr, precision))
    rtol = 1e-10 if precision == "fp64" else 1e-5
    for rank, w, cov, info in res:
        np.testing.assert_allclose(w, w_ref, rtol=rtol, atol=0)
        np.testing.assert_array_equal(cov, cov_ref)
    assert res[0][1].tobytes() == res[1][1].tobytes(), "ranks disagree"
    if precision == "fp64":   # the union graph against the oracle
        from test_gpu_pagerank import _oracle_graph_from_host
        import oracle as orc

        g = _oracle_graph_from_host(hg)
        kind = orc.trace_kinds(g)
        s = orc.power_iteration(g, orc.preference(g, kind, True))
        w_o, cov_o = orc.weights(g, s)
        np.testing.assert_allclose(w_ref, np.array(list(w_o.values())), rtol=1e-10, atol=0)
        np.testing.assert_array_equal(cov_ref, np.array(list(cov_o.values())))


def test_kind_hash_forms_agree_across_ranks():
    """Rank 0 hashes kinds with the cooperative u16 form, rank 1 with the per-thread int32 walk:
    the set hash is the same function, so the cross-rank class merge still finds every class
    (a mismatch would split classes and change the preference vector)."""
    w_ref, cov_ref = _whole(True)
    res = _run(2, True, "host", walk_ranks=(1,))
    for rank, w, cov, info in res:
        np.testing.assert_allclose(w, w_ref, rtol=1e-12, atol=0)
        np.testing.assert_array_equal(cov, cov_ref)
    assert res[0][1].tobytes() == res[1][1].tobytes(), "ranks disagree"


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_wide_op_space_int32_ids_shards(precision):
    """N = 70000 > 65535: no u16 ids, so kinds take the int32 walk and the iteration the tile
    path (fp32: config C5's precision); 2 ranks x 10k traces vs the union graph on one GPU and vs
    the oracle (fp64 restatement: 1e-10; the fp32 vectors: 1e-4, BASELINE north star)."""
    from microrank_amd import _lib
    from microrank_amd.graph import DeviceGraph
    from test_gpu_pagerank import _oracle_graph_from_host
    import oracle as orc

    n_ops, n_tr = 70_000, 10_000
    hg = _union_of_shards(n_ops, n_tr, 2)
    ctx = _lib.Context(0)
    dg = DeviceGraph.upload(ctx, hg)
    dg.pagerank(True, precision=precision)
    w_ref, cov_ref = dg.fetch()
    dg.close()
    ctx.close()
    g = _oracle_graph_from_host(hg)
    kind = orc.trace_kinds(g)
    s = orc.power_iteration(g, orc.preference(g, kind, True))
    w_o, cov_o = orc.weights(g, s)
    tol = 1e-10 if precision == "fp64" else 1e-4
    np.testing.assert_allclose(w_ref, np.array(list(w_o.values())), rtol=tol, atol=0)
    np.testing.assert_array_equal(cov_ref, np.array(list(cov_o.values())))
    res = _run(2, True, "host", big=(n_ops, n_tr, precision))
    for rank, w, cov, info in res:
        np.testing.assert_allclose(w, w_ref, rtol=1e-10 if precision == "fp64" else 1e-5, atol=0)
        np.testing.assert_array_equal(cov, cov_ref)
    assert res[0][1].tobytes() == res[1][1].tobytes(), "ranks disagree"


@pytest.mark.parametrize("tile", [False, True])
def test_empty_shard_joins_every_collective(tile):
    """Rank 1 holds no trace: it must still run every per-graph and per-iteration collective (a
    rank that returned early would leave rank 0 blocked), and both end with the whole graph's
    weights -- on the fused path and on the tile path."""
    w_ref, cov_ref = _whole(True)
    res = _run(2, True, "host", tile=tile, empty_last=True)
    for rank, w, cov, info in res:
        np.testing.assert_allclose(w, w_ref, rtol=1e-10, atol=0)
        np.testing.assert_array_equal(cov, cov_ref)
    assert res[1][3]["T"] == 0
    assert res[0][1].tobytes() == res[1][1].tobytes(), "ranks disagree"


def test_ranks_agree_on_the_iteration_path():
    """Rank 1 alone is forced onto the tile path: rank 0 must follow it (one collective protocol
    per iteration), and the result still equals the whole graph's."""
    w_ref, cov_ref = _whole(True)
    res = _run(2, True, "host", tile=(1,))
    for rank, w, cov, info in res:
        np.testing.assert_allclose(w, w_ref, rtol=1e-10, atol=0)
        np.testing.assert_array_equal(cov, cov_ref)
    assert res[0][1].tobytes() == res[1][1].tobytes(), "ranks disagree"


# ------------------------------------------------------------------ K1 over the ranks (spans)
def _span_table():
    """Spans with cross-trace duplicated spanIDs (T11 joins across the shards) and broken traces
    (orphans), 3 pods per service (pod-ops != service-ops), names=False (codes only)."""
    from microrank_amd import synth

    topo = synth.make_topology(120, 5, pods_per_service=3)
    return synth.gen_spans(topo, 6000, 9, branch=1.9, p_max=0.8, dup_span_frac=0.03, broken_frac=0.05, names=False)


def _shard_owner(st, world):
    """Rank of each trace code under SpanTable.shard(rank, world)."""
    owner = np.full(st.n_traces, -1, np.int64)
    for r in range(world):
        owner[np.unique(st.shard(r, world).trace)] = r
    return owner


def _span_mask(st):
    rng = np.random.default_rng(4)
    return (rng.random(st.n_traces) < 0.7).astype(np.uint8)


def _span_worker(rank, world, port, anomaly, q, peer=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from microrank_amd import _lib, shard
        from microrank_amd.preprocess_data import DeviceSpans

        st = _span_table()
        ctx = _lib.Context(0)
        shard.use_host(ctx)
        if peer:
            shard.use_peer(ctx)
        dev = DeviceSpans(ctx, st.shard(rank, world))
        dg = shard.build_graph(dev, _span_mask(st))
        nodes = np.array(dg.nodes)
        w, cov = shard.sharded_pagerank(dg, anomaly)
        info = dg.info()
        dg.close()
        dev.close()
        ctx.close()
        q.put((rank, w, cov, (nodes, info)))
    except Exception as e:
        q.put((rank, repr(e), None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("anomaly,world,peer", [(False, 2, False), (True, 2, False), (True, 4, False),
                                                (False, 4, True)])
def test_sharded_build_from_spans_matches_single_gpu(anomaly, world, peer):
    """Two ranks each build their graph from their own span shard (mr_graph_build_sharded: global
    node order over the ranks, T10; parent joins across the shards, T11) and rank it with
    mr_pagerank_sharded: node order equal to the single-GPU K1 graph of the whole table,
    weights within 1e-10, coverage exact, ranks bitwise, and the call-edge count of the whole
    graph.  The table has joins whose parent row lies on the other rank (counted below)."""
    import ctypes as C

    from microrank_amd import _lib
    from microrank_amd.graph import DeviceGraph
    from microrank_amd.preprocess_data import DeviceSpans
    from microrank_amd._lib import ptr

    st = _span_table()
    mask = _span_mask(st)
    sel = mask[st.trace].astype(bool)
    owner = _shard_owner(st, world)
    child_rank = owner[st.trace[sel]]
    par = st.parent[sel]
    spans_by_rank = [set(st.span[sel & (owner[st.trace] == r)].tolist()) for r in range(world)]
    cross = sum(1 for p, r in zip(par.tolist(), child_rank.tolist())
                if p >= 0 and any(p in spans_by_rank[o] for o in range(world) if o != r))
    assert cross > 0, "no cross-rank parent joins in the test table"
    ctx = _lib.Context(0)
    dev = DeviceSpans(ctx, st)
    lib = _lib.load()
    h = _lib.P()
    ctx.check(lib.mr_graph_build(ctx.h, dev.h, ptr(mask, C.c_uint8), C.byref(h)))
    info = {}
    n, t, nnz, e = C.c_int32(), C.c_int32(), C.c_int64(), C.c_int64()
    lib.mr_graph_info(h, C.byref(n), C.byref(t), C.byref(nnz), C.byref(e))
    nodes = np.empty(n.value, np.int32)
    lib.mr_graph_nodes(h, ptr(nodes, C.c_int32), ptr(np.empty(t.value, np.int32), C.c_int32))
    whole = DeviceGraph(ctx, h, nodes, None, n.value, t.value)
    whole.pagerank(anomaly)
    w_ref, cov_ref = whole.fetch()
    E_whole = e.value
    whole.close()
    dev.close()
    ctx.close()

    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_span_worker, args=(r, world, port, anomaly, q, peer)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, w, cov, extra in res:
        assert cov is not None, f"rank {rank} failed: {w}"
        np.testing.assert_array_equal(extra[0], nodes)
        np.testing.assert_allclose(w, w_ref, rtol=1e-10, atol=0)
        np.testing.assert_array_equal(cov, cov_ref)
    for r in res[1:]:
        assert r[1].tobytes() == res[0][1].tobytes(), "ranks disagree"
    assert sum(r[3][1]["T"] for r in res) == t.value
    assert res[0][3][1]["E"] == E_whole   # after the exchange: the whole graph's call edges


# ------------------------------------------------------------ peer regions over several graphs
def _seq_worker(rank, world, port, peer, q, env=None):
    """One context ranks a sequence of graphs of different op counts: the window graph (fused,
    2N + R words), a 20k-op graph (tile path, N + R words), the window graph again (smaller than
    the one before) and a 10k-op fused graph.  Every all-reduce of the sequence goes through the
    same peer region, whose arrival counts carry over from one graph to the next."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.update(env or {})
    import datetime
    import sys

    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
    k = -1
    try:
        from gpu_util import host_graph_from_oracle
        from microrank_amd import _lib, shard, synth
        from microrank_amd.graph import DeviceGraph

        ctx = _lib.Context(0)
        shard.use_host(ctx)
        if peer:
            shard.use_peer(ctx)
        win = host_graph_from_oracle(_shard(_window_graph(), rank, world))
        seq = [win, synth.big_graph(20_000, 6_000, seed=3, shard=(rank, world)), win,
               synth.big_graph(10_000, 6_000, seed=5, shard=(rank, world))]
        out = []
        for k, hg in enumerate(seq):
            print(f"[seq] rank {rank} graph {k} (N {hg.N}, T {hg.T}) peer={peer} env={env}", file=sys.stderr, flush=True)
            dg = DeviceGraph.upload(ctx, hg)
            w, cov = shard.sharded_pagerank(dg, True)
            out.append((w, cov))
            dg.close()
        ctx.close()
        q.put((rank, out, True, None))
    except Exception as e:
        print(f"[seq] rank {rank} graph {k} FAILED: {e!r}", file=sys.stderr, flush=True)
        q.put((rank, f"graph {k}: {e!r}", None, None))
    finally:
        dist.destroy_process_group()


def _run_seq(world, peer, env=None):
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_seq_worker, args=(r, world, port, peer, q, env)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    bad = [f"rank {r[0]} failed: {r[1]}" for r in res if r[2] is None]
    assert not bad, "; ".join(bad)
    return res


@pytest.mark.parametrize("mode", ["split", "fused"])
def test_peer_regions_carry_over_graphs_of_different_sizes(mode):
    """the peer all-reduce's arrival target must be the running count of pushed
    blocks, not blocks x rounds -- a smaller graph after a larger one (the window graph after the
    20k-op graph) would otherwise find its target already met and sum slots the peers had not
    written yet.  Four processes on one GPU, one context each, four graphs in sequence on the
    fused and the tile path: peer == the host-staged collective (bitwise on the fused graphs'
    exact limbs, 1e-12 on the tile path's fp64 sums) and every rank bitwise equal."""
    a = _run_seq(4, peer=False)
    b = _run_seq(4, peer=True, env={"MR_PEER_SPLIT": "1"} if mode == "split" else None)
    for k in range(4):
        for r in range(4):
            wa, ca = a[r][1][k]
            wb, cb = b[r][1][k]
            np.testing.assert_array_equal(ca, cb)
            if k == 1:
                np.testing.assert_allclose(wb, wa, rtol=1e-12, atol=0)
            else:
                assert wa.tobytes() == wb.tobytes(), f"graph {k} rank {r}: peer != host collective"
            assert b[r][1][k][0].tobytes() == b[0][1][k][0].tobytes(), "ranks disagree"


# ------------------------------------------------------------ a peer that never arrives
def _timeout_worker(rank, world, port, q, timeout_ms):
    """A sharded ranking with the peer exchange, then the same with rank 1 never signalling its
    rounds (MR_PEER_TEST_MUTE, read per call), then again unmuted: (rank, [ok times], fail time,
    error text, weights bitwise equal before / after)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MR_PEER_TIMEOUT_MS=str(timeout_ms))
    import datetime
    import time

    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
    try:
        from gpu_util import host_graph_from_oracle
        from microrank_amd import _lib, shard
        from microrank_amd.graph import DeviceGraph

        ctx = _lib.Context(0)
        shard.use_host(ctx)
        shard.use_peer(ctx)
        dg = DeviceGraph.upload(ctx, host_graph_from_oracle(_shard(_window_graph(), rank, world)))
        times, ws = [], []
        for _ in range(2):
            dist.barrier()
            ts = time.perf_counter()
            ws.append(shard.sharded_pagerank(dg, True)[0])
            times.append(time.perf_counter() - ts)
        os.environ["MR_PEER_TEST_MUTE"] = "1"
        dist.barrier()
        ts = time.perf_counter()
        err = None
        try:
            shard.sharded_pagerank(dg, True)
        except Exception as e:   # the expected outcome
            err = repr(e)
        t_fail = time.perf_counter() - ts
        os.environ.pop("MR_PEER_TEST_MUTE")
        dist.barrier()
        w_after = shard.sharded_pagerank(dg, True)[0]
        dg.close()
        ctx.close()
        q.put((rank, times, t_fail, err, ws[0].tobytes() == w_after.tobytes()))
    except Exception as e:
        q.put((rank, None, None, f"setup: {e!r}", False))
    finally:
        dist.destroy_process_group()


def test_peer_timeout_reports_within_one_timeout():
    """a rank whose rounds never arrive (two processes on one GPU, MR_PEER_TIMEOUT_MS
    = 400 ms, rank 1 muted) makes EVERY rank's sharded ranking fail with the peer-timeout error
    (agreed over the fallback collective), and the failure arrives within about one timeout -- the
    bounded spins stop on the region's error word instead of timing out again in each of the 25
    iterations (>= 10 s).  The context recovers: the next ranking (fresh regions) is bitwise the
    one before."""
    timeout_ms = 400
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_timeout_worker, args=(r, 2, port, q, timeout_ms)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, times, t_fail, err, same in res:
        assert times is not None, f"rank {rank}: {err}"
        assert err is not None and "peer timeout" in err, (rank, err)
        assert t_fail < min(times) + 3 * timeout_ms / 1e3, (rank, t_fail, times)
        assert same, f"rank {rank}: the ranking after the timeout differs"
