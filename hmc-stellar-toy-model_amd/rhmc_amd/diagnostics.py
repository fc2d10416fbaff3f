"""MCMC post-processing of gathered chains: Gelman-Rubin
R-hat, effective sample size and acceptance rates, as the reference computes
them (utils.py:86-209).  Host-side NumPy on the gathered samples — not part of
the per-step hot path."""
import numpy as np


def variogram(chains, var_num, t_lag):
    """utils.py:170-188 (BDA eq. 11.7)."""
    m = len(chains)
    n = chains[0].shape[0]
    V_t = 0.
    for i in range(m):
        c = chains[i][:, var_num]
        V_t += np.sum(np.square(c[t_lag:] - c[:-t_lag]))
    return V_t / float(m * (n - t_lag))


def convergence_stats(q_chain, thin_rate=5, warm_up_num=0):
    """utils.py:86-168: (R_hat[D], n_eff[D]) of q_chain [Nchain, Niter, D];
    each chain is warmed up, thinned, trimmed to even length and split in two.
    `n = L_chain/2` is Python 2 integer division in the reference."""
    Nchain, Niter, D = q_chain.shape
    assert Nchain > 1
    chains = []
    for mm in range(Nchain):
        c = q_chain[mm, warm_up_num:, :][::thin_rate, :]
        L = c.shape[0]
        if L % 2:
            c = c[:L - 1]
        n = L // 2
        chains.append(c[:n])
        chains.append(c[n:])
    m = len(chains)
    W = np.mean(np.array([np.std(c, ddof=1, axis=0) for c in chains]), axis=0)
    mean_within = np.array([np.mean(c, axis=0) for c in chains])
    mean_all = np.mean(mean_within, axis=0)
    B = np.sum(np.square(mean_within - mean_all), axis=0) * n / float(m - 1)
    var = W * (n - 1) / float(n) + B / float(n)
    R = np.sqrt(var / W)
    n_eff = np.zeros(D, dtype=float)
    for i in range(D):
        rho_t1 = 1. - variogram(chains, i, 1) / (2 * var[i])
        rho_t2 = 1. - variogram(chains, i, 2) / (2 * var[i])
        if rho_t1 < 5e-2:
            sum_rho = 0
        else:
            rho_t = [rho_t1, rho_t2]
            t = 1
            while t < n - 2:
                rho_t.append(1 - variogram(chains, i, t + 2) / (2 * var[i]))
                if ((t % 2) == 1) & ((rho_t[t] + rho_t[t + 1]) < 0):
                    break
                t += 1
            sum_rho = np.sum(rho_t[:t])
            if sum_rho < 0:
                sum_rho = 0
        n_eff[i] = m * n / (1 + 2 * sum_rho)
    return R, n_eff


def acceptance_rate(decision_chain, start=None, end=None):
    """utils.py:192-209: decision_chain [Nchain, Niter, 1] of 0/1."""
    _, Niter, _ = decision_chain.shape
    if start is None and end is None:
        return np.sum(decision_chain, axis=(1, 2)) / Niter
    Niter = end - start if end > 0 else Niter - start
    return np.sum(decision_chain[:, start:end, :], axis=(1, 2)) / Niter
