"""Simulator (drop-in for simulator.py:12-201).

Owns the data, the workers and f(x*), runs the four trainers in the reference's
order over ONE shared numpy RNG stream (Centralized, Ring, Grid when N is a
perfect square, Fully Connected; simulator.py:94-137), records
iterations-to-threshold and floats transmitted, prints and plots.  The trainers
underneath run on the GPU (trainer.py in this package); the reference optimum
still comes from sklearn's saga solver like upstream (simulator.py:32-69).
"""
import numpy as np
from sklearn.linear_model import LogisticRegression as SklearnLogisticRegression
from sklearn.linear_model import Ridge as SklearnRidge

from obj_problems import logistic_objective, quadratic_objective
from trainer import CentralizedTrainer, DecentralizedTrainer
from utils import generate_and_preprocess_data
from worker import Worker


class Simulator:
    def __init__(self, config):
        self.config = config
        self.worker_data, self.n_features, self.X_full, self.y_full = \
            generate_and_preprocess_data(config["n_workers"], config)
        self.workers = self._create_workers()
        self.f_opt = self._compute_reference_optimum()
        self.results = {}
        self.numerical_results = {}

    def _create_workers(self):
        c = self.config
        return [Worker(i, self.worker_data[i], c["local_batch_size"], self.n_features, c)
                for i in range(c["n_workers"])]

    def _reset_workers(self):
        self.workers = self._create_workers()

    def _compute_reference_optimum(self):
        kind = self.config["problem_type"]
        reg = self.config["l2_regularization_lambda"]
        X_nb, y = self.X_full[:, :-1], self.y_full
        alpha = reg * self.X_full.shape[0]
        if kind == "logistic":
            solver = SklearnLogisticRegression(penalty="l2", C=1.0 / alpha if alpha > 1e-12 else 1e12,
                                               fit_intercept=True, solver="saga", max_iter=5000, tol=1e-9,
                                               random_state=42)
            solver.fit(X_nb, y)
            w_opt = np.concatenate([solver.coef_.flatten(), solver.intercept_])
            f = logistic_objective(w_opt, self.X_full, self.y_full, reg)
        elif kind == "quadratic":
            solver = SklearnRidge(alpha=alpha, fit_intercept=True, solver="saga", max_iter=5000, tol=1e-9,
                                  random_state=42)
            solver.fit(X_nb, y)
            w_opt = np.concatenate([solver.coef_.flatten(), [solver.intercept_]])
            f = quadratic_objective(w_opt, self.X_full, self.y_full, reg)
        else:
            raise ValueError("Unknown problem type")
        print(f"Ref f(x*) calculated: {f:.6f}")
        return f

    def _record_numerical_results(self, label, history, trainer):
        threshold = self.config.get("suboptimality_threshold", 0.05)
        obj = np.array(history.get("objective", []))
        iters = -1
        if len(obj) > 0:
            hit = np.where(obj <= threshold)[0]
            if len(hit) > 0:
                iters = hit[0] + 1
        total = getattr(trainer, "total_floats_transmitted", 0)
        n = self.config["n_workers"]
        self.numerical_results[label] = {
            "iterations_to_threshold": iters,
            "total_transmission_floats": total,
            "avg_worker_transmission_floats": total / n if n > 0 else 0,
        }

    def _run_one(self, label, make_trainer):
        self._reset_workers()
        trainer = make_trainer()
        if label is None:  # grid: label from the trainer (simulator.py:113)
            label = f"D-SGD ({trainer.topology.capitalize()})"
        hist, _ = trainer.run(self.config["n_iterations"], self.X_full, self.y_full, self.f_opt)
        self.results[label] = hist
        self._record_numerical_results(label, hist, trainer)

    def run_all(self):
        c = self.config
        print(f"\n=== Starting Simulation: {c['problem_type']} ===")
        self._run_one("Centralized", lambda: CentralizedTrainer(self.workers, self.n_features, c))
        self._run_one("D-SGD (Ring)", lambda: DecentralizedTrainer(self.workers, "ring", self.n_features, c))
        n = c["n_workers"]
        if int(np.sqrt(n)) ** 2 == n and n > 0:
            self._run_one(None, lambda: DecentralizedTrainer(self.workers, "grid", self.n_features, c))
        else:
            print("\nSkipping Grid topology: N_WORKERS is not perfect square")
            self.numerical_results["D-SGD (Grid)"] = {"iterations_to_threshold": "N/A",
                                                      "total_transmission_floats": "N/A",
                                                      "avg_worker_transmission_floats": "N/A"}
        self._run_one("D-SGD (Fully Connected)",
                      lambda: DecentralizedTrainer(self.workers, "fully_connected", self.n_features, c))
        print("\n=== Simulation Finished ===")
        self.report_numerical_results()

    @staticmethod
    def _order(labels):
        return sorted(labels, key=lambda x: (not x.startswith("Centralized"), x))

    def report_numerical_results(self):
        print("\n--- Numerical Results ---")
        thr = self.config.get("suboptimality_threshold", 0.07)
        print(f"Target Suboptimality Gap Threshold: {thr}")
        labels = self._order(self.numerical_results.keys())
        width = max(len(s) for s in labels) + 2 if labels else 2
        print(f"\nIterations to reach suboptimality gap <= {thr}:")
        for lab in labels:
            it = self.numerical_results[lab]["iterations_to_threshold"]
            if it == "N/A":
                print(f"  {lab:<{width}}: N/A")
            elif it == -1:
                print(f"  {lab:<{width}}: > {self.config['n_iterations']} , threshold not reached")
            else:
                print(f"  {lab:<{width}}: {it} iterations")
        print(f"\nTotal Data Transmission in floats, over {self.config['n_iterations']} iterations:")
        for lab in labels:
            r = self.numerical_results[lab]
            if r["total_transmission_floats"] == "N/A":
                print(f"  {lab:<{width}}: Total = N/A, Avg per Worker = N/A")
            else:
                print(f"  {lab:<{width}}: Total = {r['total_transmission_floats']:.3e}, "
                      f"Avg per Worker = {r['avg_worker_transmission_floats']:.3e}")

    def plot_results(self, show=True):
        import matplotlib.pyplot as plt

        c = self.config
        T = c["n_iterations"]
        its = np.arange(1, T + 1)
        panels = [("objective", f"Suboptimality Gap ($f(\\bar{{x}}_T) - f(x^*)$) - {c['problem_type']}"),
                  ("consensus_error",
                   f"Consensus Error ($(1/N) \\sum ||x_{{i,T}} - \\bar{{x}}_T||^2$) - {c['problem_type']}")]
        plt.figure(figsize=(7 * len(panels), 6))
        for k, (key, title) in enumerate(panels, 1):
            ax = plt.subplot(1, len(panels), k)
            for lab in self._order(self.results.keys()):
                hist = self.results.get(lab)
                if not hist or key not in hist or (key == "consensus_error" and lab == "Centralized"):
                    continue
                data = hist[key]
                if len(data) != T:
                    print(f"Warning: Mismatched data length for metric '{key}' in '{lab}'. "
                          f"Expected {T}, got {len(data)}. Skipping.")
                    continue
                v = np.array(data)
                if np.any(~np.isfinite(v)):
                    print(f"Warning: Non-finite values found in metric '{key}' for '{lab}'. Skipping plot line.")
                    continue
                ax.plot(its, np.maximum(v, 1e-14), label=lab, lw=2)
            ax.set_xlabel("Iteration (T)")
            ax.set_ylabel("Value (log scale)")
            ax.set_yscale("log")
            ax.set_title(title)
            ax.grid(True, which="both", linestyle="--", linewidth=0.5)
            ax.legend()
        plt.figtext(0.5, 0.01,
                    f"Config: N={c['n_workers']}, b={c['local_batch_size']}, Problem={c['problem_type']}, "
                    f"Non-IID Data, LR0={c['learning_rate_eta0']} (Sqrt Decay), "
                    f"$\\lambda$={c['l2_regularization_lambda']}", ha="center", fontsize=10)
        plt.tight_layout(rect=[0, 0.05, 1, 0.97])
        if show:
            plt.show()
