"""Does the C3 round kernel start slow after the GPU idles?  Run under rocprofv3 --kernel-trace:
segment A = 40 rounds after a 0.5 s host pause, segment B = 40 rounds right after A."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import _dopt  # noqa: E402
import topology as TP  # noqa: E402

n, d, m = 4096, 1024, 512
eng = _dopt.Engine(0, "float64", data_dtype="float32")
top = TP.random_regular(n, 4, seed=0)
eng.generate_shards("logistic", n, d, m, seed=1000, flip=0.05)
eng.set_topology(top.row_ptr, top.col, top.w)
eng.set_models(np.zeros((n, d)))
eng.run_dsgd_pipelined(5, 0.05, m, 1e-4, 1e-4, 0.0)
eng.sync()
time.sleep(0.5)
eng.run_dsgd_pipelined(40, 0.05, m, 1e-4, 1e-4, 0.0)  # segment A
eng.run_dsgd_pipelined(40, 0.05, m, 1e-4, 1e-4, 0.0)  # segment B
eng.run_dsgd_pipelined(0, 0.05, m, 1e-4, 1e-4, 0.0)
eng.sync()
eng.close()
