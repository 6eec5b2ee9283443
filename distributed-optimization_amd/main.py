"""Entry point (drop-in for main.py): the report's N=25 experiment on the GPU engine.

Same module constants and seed as the reference (main.py:6-24).  Run from this
directory:  python main.py
"""
import numpy as np

from simulator import Simulator

N_WORKERS = 25
LOCAL_BATCH_SIZE = 16
N_ITERATIONS = 10000
LEARNING_RATE_ETA0 = 0.05
SUBOPTIMALITY_THRESHOLD = 0.08

PROBLEM_TYPE = "quadratic"  # 'logistic', 'quadratic'

N_SAMPLES = N_WORKERS * 500
N_FEATURES = 80
N_INFORMATIVE_FEATURES = 50
CLASSIFICATION_SEP = 0.7

L2_REGULARIZATION_LAMBDA = 1e-4
STRONG_CONVEXITY_MU = L2_REGULARIZATION_LAMBDA


def make_config(**overrides):
    cfg = {
        "n_workers": N_WORKERS,
        "local_batch_size": LOCAL_BATCH_SIZE,
        "n_iterations": N_ITERATIONS,
        "learning_rate_eta0": LEARNING_RATE_ETA0,
        "l2_regularization_lambda": L2_REGULARIZATION_LAMBDA,
        "strong_convexity_mu": STRONG_CONVEXITY_MU,
        "problem_type": PROBLEM_TYPE,
        "n_samples": N_SAMPLES,
        "n_features": N_FEATURES,
        "n_informative_features": N_INFORMATIVE_FEATURES,
        "classification_sep": CLASSIFICATION_SEP,
        "suboptimality_threshold": SUBOPTIMALITY_THRESHOLD,
    }
    cfg.update(overrides)
    return cfg


def _maybe_init_distributed():
    """Under torch.distributed.run (WORLD_SIZE > 1) every rank runs this script; the
    trainers then split the workers across the ranks' GPUs (trainer.py docstring), every rank
    computes the same histories, and rank 0 alone prints the report and plots (the reference's
    single process prints it once).  Returns True on the rank that reports."""
    import os

    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        if int(os.environ.get("RANK", "0")) != 0:
            import sys

            sys.stdout = open(os.devnull, "w")
        import torch

        import distributed

        local = int(os.environ.get("DOPT_DEVICE", os.environ.get("LOCAL_RANK", "0")))  # (trainer._device)
        torch.cuda.set_device(local)
        distributed.init_process_group(os.environ.get("DOPT_BACKEND", "nccl"))
        return int(os.environ.get("RANK", "0")) == 0
    return True


def _finish_distributed():
    """The engine's RCCL communicators (devices drained, engines detached), then the process group."""
    import os

    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch.distributed as dist

        import distributed

        distributed.close_comms()
        dist.destroy_process_group()


if __name__ == "__main__":
    reporter = _maybe_init_distributed()
    np.random.seed(203)
    simulator = Simulator(make_config())
    simulator.run_all()
    if reporter:
        simulator.plot_results()
    _finish_distributed()
