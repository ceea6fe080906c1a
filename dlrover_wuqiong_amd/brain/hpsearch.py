"""Hyper-parameter search: Gaussian-process Bayesian optimisation.

``BayesianOptimizer(bounds, history, num_candidates, use_variance)`` proposes
``num_candidates`` points: uniform random ones on a cold start, otherwise it
fits a GP (Matern-5/2 ARD kernel on inputs normalised to the unit cube,
standardised outcomes; length-scales / signal / noise by maximising the log
marginal likelihood with L-BFGS-B from several starts) and maximises
Expected Improvement (noisy EI = EI over the posterior-mean incumbent with
the observed per-point noise when ``use_variance``).  A batch of q points is
built greedily with the "kriging believer" heuristic: each chosen point is
added to the GP at its posterior mean before the next one is picked.

numpy + scipy only (the reference uses botorch/gpytorch, which are not part
of this stack).  Rewards are MAXIMISED.

Parity: reference ``dlrover/python/brain/hpsearch/base.py`` (``RunResult``,
``OptimizerBase``) and ``hpsearch/bo.py`` (``BayesianOptimizer``).
"""

import math
from abc import ABC, abstractmethod
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
from scipy.optimize import minimize
from scipy.stats import norm


@dataclass
class RunResult:
    parameters: Tuple = ()
    reward: float = 0.0
    variance: float = 0.01
    epsilon: float = 0.0


class OptimizerBase(ABC):
    def __init__(self, bounds: Sequence[Sequence[float]], history: List[List[RunResult]], num_candidates: int,
                 seed: Optional[int] = None, **kwargs):
        self.bounds = [tuple(map(float, b)) for b in bounds]
        self.history = history or []
        self.num_candidates = num_candidates
        self.cold_start = len(sum(self.history, [])) == 0
        self.rng = np.random.default_rng(seed)

    @abstractmethod
    def optimize(self) -> List[RunResult]:
        pass

    def _random(self, n: int) -> np.ndarray:
        lo = np.array([b[0] for b in self.bounds])
        hi = np.array([b[1] for b in self.bounds])
        return lo + (hi - lo) * self.rng.random((n, len(self.bounds)))


class RandomSearch(OptimizerBase):
    def optimize(self) -> List[RunResult]:
        return [RunResult(parameters=tuple(x)) for x in self._random(self.num_candidates).tolist()]


def _matern52(a: np.ndarray, b: np.ndarray, ls: np.ndarray) -> np.ndarray:
    d = np.sqrt(np.maximum(((a[:, None, :] - b[None, :, :]) / ls) ** 2, 0).sum(-1))
    s5 = math.sqrt(5.0) * d
    return (1.0 + s5 + 5.0 / 3.0 * d * d) * np.exp(-s5)


class GaussianProcess:
    """Exact GP regression (zero mean on standardised targets)."""

    def __init__(self, x: np.ndarray, y: np.ndarray, noise: Optional[np.ndarray] = None, restarts: int = 4,
                 rng: Optional[np.random.Generator] = None):
        self.x = x
        self.y_mean, self.y_std = float(y.mean()), float(y.std() or 1.0)
        self.y = (y - self.y_mean) / self.y_std
        self.fixed_noise = None if noise is None else np.maximum(noise / self.y_std ** 2, 1e-6)
        self.rng = rng or np.random.default_rng(0)
        self._fit(restarts)

    def _nll(self, theta: np.ndarray) -> float:
        d = self.x.shape[1]
        ls, sf2 = np.exp(theta[:d]), np.exp(theta[d])
        noise = self.fixed_noise if self.fixed_noise is not None else np.exp(theta[d + 1]) * np.ones(len(self.y))
        k = sf2 * _matern52(self.x, self.x, ls) + np.diag(noise + 1e-8)
        try:
            L = np.linalg.cholesky(k)
        except np.linalg.LinAlgError:
            return 1e10
        alpha = np.linalg.solve(L.T, np.linalg.solve(L, self.y))
        # weak log-normal prior on length-scales keeps tiny data sets sane
        prior = 0.5 * ((theta[:d] - np.log(0.5)) ** 2).sum()
        return float(0.5 * self.y @ alpha + np.log(np.diag(L)).sum() + prior)

    def _fit(self, restarts: int):
        d = self.x.shape[1]
        n_theta = d + 1 + (0 if self.fixed_noise is not None else 1)
        best, best_v = None, np.inf
        bounds = [(np.log(1e-2), np.log(10.0))] * d + [(np.log(1e-2), np.log(10.0))]
        if self.fixed_noise is None:
            bounds.append((np.log(1e-6), np.log(1.0)))
        for r in range(restarts):
            x0 = np.zeros(n_theta)
            x0[:d] = np.log(0.5) if r == 0 else self.rng.uniform(np.log(0.05), np.log(2.0), d)
            if self.fixed_noise is None:
                x0[-1] = np.log(1e-2)
            res = minimize(self._nll, x0, method="L-BFGS-B", bounds=bounds)
            if res.fun < best_v:
                best, best_v = res.x, res.fun
        self.theta = best
        ls, sf2 = np.exp(best[:d]), np.exp(best[d])
        noise = self.fixed_noise if self.fixed_noise is not None else np.exp(best[d + 1]) * np.ones(len(self.y))
        self.ls, self.sf2, self.noise = ls, sf2, noise
        k = sf2 * _matern52(self.x, self.x, ls) + np.diag(noise + 1e-8)
        self.L = np.linalg.cholesky(k)
        self.alpha = np.linalg.solve(self.L.T, np.linalg.solve(self.L, self.y))

    def predict(self, xs: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        ks = self.sf2 * _matern52(xs, self.x, self.ls)
        mu = ks @ self.alpha
        v = np.linalg.solve(self.L, ks.T)
        var = np.maximum(self.sf2 - (v * v).sum(0), 1e-12)
        return mu, np.sqrt(var)


def expected_improvement(mu: np.ndarray, sd: np.ndarray, best: float, xi: float = 0.0) -> np.ndarray:
    z = (mu - best - xi) / sd
    return (mu - best - xi) * norm.cdf(z) + sd * norm.pdf(z)


class BayesianOptimizer(OptimizerBase):
    NUM_RESTARTS = 5
    RAW_SAMPLES = 512

    def __init__(self, bounds, history, num_candidates, use_variance: bool = False, seed: Optional[int] = None,
                 **kwargs):
        super().__init__(bounds, history, num_candidates, seed=seed, **kwargs)
        self.use_variance = use_variance

    def _unit(self, x: np.ndarray) -> np.ndarray:
        lo = np.array([b[0] for b in self.bounds])
        hi = np.array([b[1] for b in self.bounds])
        return (x - lo) / np.where(hi > lo, hi - lo, 1.0)

    def _from_unit(self, u: np.ndarray) -> np.ndarray:
        lo = np.array([b[0] for b in self.bounds])
        hi = np.array([b[1] for b in self.bounds])
        return lo + u * (hi - lo)

    def optimize(self) -> List[RunResult]:
        if self.cold_start:
            return [RunResult(parameters=tuple(x)) for x in self._random(self.num_candidates).tolist()]
        runs = sum(self.history, [])
        x = self._unit(np.array([r.parameters for r in runs], dtype=np.float64))
        y = np.array([float(r.reward) for r in runs], dtype=np.float64)
        noise = np.array([float(r.variance) for r in runs]) if self.use_variance else None
        d = x.shape[1]
        chosen: List[np.ndarray] = []
        for _ in range(self.num_candidates):
            gp = GaussianProcess(x, y, noise, rng=self.rng)
            mu_obs, _ = gp.predict(x)
            # noisy EI: improve over the best posterior mean at observed points
            best = float(mu_obs.max()) if self.use_variance else float(gp.y.max())

            def neg_ei(u):
                m, s = gp.predict(np.atleast_2d(u))
                return -float(expected_improvement(m, s, best)[0])

            raw = self.rng.random((self.RAW_SAMPLES, d))
            m, s = gp.predict(raw)
            ei = expected_improvement(m, s, best)
            starts = raw[np.argsort(-ei)[:self.NUM_RESTARTS]]
            best_u, best_v = starts[0], -np.inf
            for s0 in starts:
                res = minimize(neg_ei, s0, method="L-BFGS-B", bounds=[(0.0, 1.0)] * d)
                if -res.fun > best_v:
                    best_u, best_v = np.clip(res.x, 0, 1), -res.fun
            chosen.append(best_u)
            # kriging believer: pretend we observed the posterior mean there
            mb, _ = gp.predict(best_u[None])
            x = np.vstack([x, best_u[None]])
            y = np.append(y, mb[0] * gp.y_std + gp.y_mean)
            if noise is not None:
                noise = np.append(noise, float(np.median(noise)))
        return [RunResult(parameters=tuple(self._from_unit(u).tolist())) for u in chosen]
