"""Engine's own HIP stream vs a torch stream for the fused C3 round (float64 over float32 rows):
order alternated per repetition, a warm-up call before each measured call; HIP-event kernel
averages and wall time per round."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _dopt  # noqa: E402
import topology as TP  # noqa: E402


def main():
    n, d, m, K = 4096, 1024, 512, int(os.environ.get("AB_STEPS", "40"))
    eng = _dopt.Engine(0, "float64", data_dtype="float32")
    eng.generate_shards("logistic", n, d, m, seed=1000, flip=0.05)
    top = TP.random_regular(n, 4, seed=0)
    eng.set_topology(top.row_ptr, top.col, top.w)
    ts = torch.cuda.Stream()
    hp = torch.cuda.Stream(priority=-1)
    streams = {"own": 0, "torch": ts.cuda_stream, "torch_hi": hp.cuda_stream}
    res = {}
    eng.set_models(np.zeros((n, d)))
    for rep in range(4):
        order = list(streams) if rep % 2 == 0 else list(reversed(list(streams)))
        for name in order:
            eng.set_stream(streams[name])
            eng.run_dsgd_pipelined(10, 0.05, m, 1e-4, 1e-4, 0.0)  # warm-up (continues the chain)
            eng.kernel_stats()
            eng.set_profiling(True, every=1)
            eng.sync()
            t = time.perf_counter()
            eng.run_dsgd_pipelined(K, 0.05, m, 1e-4, 1e-4, 0.0)
            eng.sync()
            dt = (time.perf_counter() - t) / K * 1e3
            k, ms = eng.kernel_stats()
            eng.set_profiling(False)
            eng.run_dsgd_pipelined(0, 0.05, m, 1e-4, 1e-4, 0.0)
            res.setdefault(name, []).append((ms / k, dt))
            print(f"rep {rep} {name:9s} kernel {ms / k:.4f} ms  round {dt:.4f} ms", flush=True)
        eng.set_stream(0)
    for k, v in res.items():
        a = sorted(x for x, _ in v)
        b = sorted(y for _, y in v)
        print(k, "kernel best %.4f median %.4f | round best %.4f median %.4f" % (a[0], a[len(a) // 2], b[0],
                                                                                 b[len(b) // 2]))
    eng.close()


if __name__ == "__main__":
    main()
