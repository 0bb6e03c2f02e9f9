"""Helpers shared by the GPU tests: oracle graphs -> product host graphs, golden -> dicts."""
import numpy as np

import oracle as orc
from microrank_amd.graph import HostGraph, _csr


def host_graph_from_oracle(g: "orc.Graph") -> HostGraph:
    N, T = g.N, g.T
    sr_off, sr_ops = _csr(g.sr_t, g.sr_o, T, N)
    rs_off, rs_ops = _csr(g.rs_t, g.rs_o, T, N)
    same = np.array_equal(sr_off, rs_off) and np.array_equal(sr_ops, rs_ops)
    ss_off, ss_par = _csr(g.ss_c, g.ss_p, N, N)
    ident = np.array_equal(g.pr_idx, np.arange(T)) and np.array_equal(g.pr_len, g.len_t)
    return HostGraph(list(g.nodes), list(g.traces), sr_off, sr_ops, None if same else rs_off,
                     None if same else rs_ops, g.len_t.astype(np.int32), g.len_o.astype(np.int32), ss_off,
                     ss_par, g.nchild.astype(np.int32), None if ident else g.pr_idx.astype(np.int32),
                     None if ident else g.pr_len.astype(np.int32))


def golden_graph_dicts(exp, tnames):
    """Compact golden graph (make_golden.dump_graph) -> the four reference dicts."""
    nodes = exp["nodes"]

    def unflat(d, kname, vname):
        out = {}
        pos = 0
        for k, ln in zip(d["keys"], d["len"]):
            out[kname(k)] = [vname(v) for v in d["vals"][pos:pos + ln]]
            pos += ln
        return out

    oo = unflat(exp["operation_operation"], lambda i: nodes[i], lambda i: nodes[i])
    ot = unflat(exp["operation_trace"], lambda i: tnames[i], lambda i: nodes[i])
    to = unflat(exp["trace_operation"], lambda i: nodes[i], lambda i: tnames[i])
    return oo, ot, to, dict(ot)


def c2_graph(n_ops=1000, n_traces=200_000, seed=7, anomaly_split=True):
    """A C2-shaped window graph built by the oracle from synthetic spans."""
    from microrank_amd import synth

    topo = synth.make_topology(n_ops, seed)
    st = synth.gen_spans(topo, n_traces, seed + 1, branch=1.9, p_max=0.8, names=False)
    sel = np.ones(n_traces, dtype=bool)
    sg = orc.span_graph(st.trace, st.podop, st.span, st.parent, sel)
    return st, sg
