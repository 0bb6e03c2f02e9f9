import sys, os
sys.path[:0]=['.','oracle','tests']
import numpy as np
from microrank_amd import _lib
from microrank_amd.pagerank import trace_pagerank
for mode in ["0","1"]:
    os.environ["MR_TRACE_MODE"]=mode
    try:
        print(mode, trace_pagerank({"a":["b"],"b":[]},{"t":["a","b"],"u":["b"]},{"a":["t"],"b":["t","u"]},{"t":["a","b"],"u":["b"]},True))
    except Exception as e:
        print(mode, "ERR", e)
