"""Why is the phase path's gradient kernel slower than the fused round kernel?  C3 (float64 over
float32 rows) on one engine, round-kernel averages by HIP events, interleaved repetitions:
  fused/own    dopt_run_dsgd_pipelined on the engine's own stream
  fused/torch  the same on a torch stream (dopt_set_stream), as the phase path runs
  grad/loss    dopt_phase_grad (F_GOUT) with the loss at xbar, on the torch stream
  grad/none    dopt_phase_grad without metrics"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _dopt  # noqa: E402
import topology as TP  # noqa: E402


def main():
    n, d, m, K = 4096, 1024, 512, int(os.environ.get("AB_STEPS", "20"))
    eng = _dopt.Engine(0, "float64", data_dtype="float32")
    eng.generate_shards("logistic", n, d, m, seed=1000, flip=0.05)
    top = TP.random_regular(n, 4, seed=0)
    eng.set_topology(top.row_ptr, top.col, top.w)
    own = None
    ts = torch.cuda.Stream()
    res = {}

    def timed(name, fn):
        eng.kernel_stats()
        eng.set_profiling(True, every=1)
        fn()
        eng.sync()
        k, ms = eng.kernel_stats()
        eng.set_profiling(False)
        res.setdefault(name, []).append(ms / k)
        print(f"{name:12s} {ms / k:.4f} ms ({k} launches) [{_dopt.last_round_kernel()}]", flush=True)

    def fused():
        eng.run_dsgd_pipelined(K, 0.05, m, 1e-4, 1e-4, 0.0)
        eng.run_dsgd_pipelined(0, 0.05, m, 1e-4, 1e-4, 0.0)

    def grad(flags):
        def f():
            eng.phase_begin(m)
            for _ in range(K):
                eng.phase_grad(m, 1e-4, flags)
        return f

    ld, _ = eng.layout()
    sums = torch.zeros(ld, dtype=torch.float64, device="cuda")

    def sched():  # the lagged phase schedule at world 1: colsum (+ fold) -> grad (+ loss) -> mix
        eng.phase_begin(m)
        eng.phase_gather()
        for h in range(K):
            eng.phase_colsum_fold(sums.data_ptr())
            eng.phase_grad(m, 1e-4, _dopt.RUN_OBJECTIVE if h >= 2 else 0)
            eng.phase_mix_lagged(h, 0.05, sums.data_ptr(), True)

    for rep in range(3):
        eng.set_models(np.zeros((n, d)))
        if own is None:
            timed("fused/own", fused)
            own = True
        else:
            timed("fused/own", fused)
        eng.set_stream(ts.cuda_stream)
        timed("fused/torch", fused)
        timed("grad/loss", grad(_dopt.RUN_OBJECTIVE))  # at the iterate the fused rounds left
        x_now = eng.get_models()
        eng.set_models(np.zeros((n, d)))
        timed("grad/loss0", grad(_dopt.RUN_OBJECTIVE))  # at zero iterates
        eng.set_models(x_now)
        timed("grad/none", grad(0))
        timed("grad/both", grad(_dopt.RUN_OBJECTIVE | _dopt.RUN_CONSENSUS))
        with torch.cuda.stream(ts):
            timed("sched", sched)
        eng.set_stream(0)
    for k, v in res.items():
        print(k, "best %.4f median %.4f" % (min(v), sorted(v)[len(v) // 2]))
    eng.close()


if __name__ == "__main__":
    main()
