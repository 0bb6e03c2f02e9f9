"""Host phases of the drop-in window body (online_rca.py:167-201 through the swapped imports) at C2:
wall time per call of each drop-in function over a few windows, then a cProfile of one window
(top entries by cumulative time).  GPU box:  python3 scripts/dropin_phases.py [n_windows]"""
import contextlib
import cProfile
import io
import os
import pstats
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import pandas as pd  # noqa: E402

from microrank_amd import synth  # noqa: E402
from microrank_amd import online_rca as orca  # noqa: E402
from microrank_amd.preprocess_data import get_operation_slo, get_service_operation_list  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    ndf, adf = synth.window_dataframes(1000, 200_000, 1234, branch=1.9, p_max=0.8, fault_ms=6000.0)
    op_list = get_service_operation_list(ndf)
    slo = get_operation_slo(op_list, ndf)
    start = adf["startTime"].min()
    one = start + pd.Timedelta(1, unit="ns")
    acc = {}

    def timed(name, fn):
        def w(*a, **k):
            ts = time.perf_counter()
            r = fn(*a, **k)
            acc.setdefault(name, []).append((time.perf_counter() - ts) * 1e3)
            return r
        return w

    names = ("system_anomaly_detect", "get_pagerank_graph", "trace_pagerank", "calculate_spectrum_without_delay_list",
             "_write_result")
    orig = {k: getattr(orca, k) for k in names}
    for k in names:
        setattr(orca, k, timed(k, orig[k]))
    td = tempfile.mkdtemp(dir="/tmp")
    os.chdir(td)
    with contextlib.redirect_stdout(io.StringIO()):
        ts = time.perf_counter()
        orca._window_loop(adf, slo, op_list, start, one)
        first = (time.perf_counter() - ts) * 1e3
    acc.clear()
    walls = []
    for _ in range(n):
        with contextlib.redirect_stdout(io.StringIO()):
            ts = time.perf_counter()
            orca._window_loop(adf, slo, op_list, start, one)
            walls.append((time.perf_counter() - ts) * 1e3)
    print(f"first window {first:.1f} ms; later windows (ms): {[round(x, 2) for x in walls]}")
    for k in names:
        v = acc.get(k, [])
        print(f"  {k:40s} calls/window {len(v) / n:3.0f}  ms/window {sum(v) / n:8.3f}")
    for k in names:
        setattr(orca, k, orig[k])
    pr = cProfile.Profile()
    with contextlib.redirect_stdout(io.StringIO()):
        pr.enable()
        orca._window_loop(adf, slo, op_list, start, one)
        pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(40)
    print(s.getvalue())


if __name__ == "__main__":
    main()
