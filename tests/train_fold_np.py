"""float64 numpy restatement of the opt-in train-mode affine fold (pc-nerf_amd/csrc/nof_fold.hip) -- test
infrastructure only, the checker of the HIP kernels' algebra.

One BatchNorm chunk of the reference NOF in train mode (nof/networks/models.py:183-203, every LeakyReLU(True) the
identity: models.py:72,152,232) is sigmoid(a . e + c) with (a, c) composed from the chunk's encoding mean and
covariance; the backward is the hand-derived adjoint the kernels implement (k_tf_bwd_out / k_tf_bwd_layer /
k_tf_dw), checked here against torch float64 autograd of the layer-by-layer network.
"""
import numpy as np

from nof import synthetic as syn


def _p(params, key):
    return np.asarray(params[key], dtype=np.float64)


def fold_forward(params, e, eps=1e-5):
    """-> (a (63,), c, state) for one chunk of encodings e (n, 63); state holds the per-layer maps and the
    BatchNorm batch statistics (mean of h_L, biased variance) for the running-stat update."""
    lin, bn = syn.nof_param_names()
    e = np.asarray(e, dtype=np.float64)
    n = len(e)
    eb = e.mean(0)
    d = e - eb
    S = d.T @ d / n
    maps, P, beta_prev = [], None, None
    for L in range(8):
        W, b = _p(params, lin[L] + ".weight"), _p(params, lin[L] + ".bias")
        gamma, beta = _p(params, bn[L] + ".weight"), _p(params, bn[L] + ".bias")
        if L == 0:
            Pp, mean = W.copy(), W @ eb + b
        elif L == 4:
            Pp, mean = W[:, :63] + W[:, 63:] @ P, W[:, :63] @ eb + W[:, 63:] @ beta_prev + b
        else:
            Pp, mean = W @ P, W @ beta_prev + b
        Q = Pp @ S
        v = np.einsum("ij,ij->i", Q, Pp)
        r = 1.0 / np.sqrt(v + eps)
        s = gamma * r
        maps.append(dict(Pp=Pp, Q=Q, var=v, r=r, s=s, mean=mean, gamma=gamma, W=W))
        P, beta_prev = s[:, None] * Pp, beta
    w = _p(params, "occ_out.0.weight")[0]
    a = w @ P
    c = float(w @ beta_prev + _p(params, "occ_out.0.bias")[0] - a @ eb)
    return a, c, dict(eb=eb, S=S, n=n, maps=maps)


def running_update(params, state, momentum=0.1):
    """nn.BatchNorm1d's running-stat update for this chunk (unbiased variance), in place on ``params``."""
    _, bn = syn.nof_param_names()
    n = state["n"]
    for L, m in enumerate(state["maps"]):
        rm, rv = bn[L] + ".running_mean", bn[L] + ".running_var"
        params[rm] = (momentum * m["mean"] + (1 - momentum) * _p(params, rm)).astype(np.float32)
        params[rv] = (momentum * m["var"] * n / (n - 1) + (1 - momentum) * _p(params, rv)).astype(np.float32)


def fold_backward(params, e, g, state):
    """Parameter gradients (state_dict keys) of sum_s L(logit_s) given g = dL/dlogit per row of e."""
    lin, bn = syn.nof_param_names()
    e = np.asarray(e, dtype=np.float64)
    g = np.asarray(g, dtype=np.float64)
    eb, maps = state["eb"], state["maps"]
    abar, gbar = (e - eb).T @ g, g.sum()
    w = _p(params, "occ_out.0.weight")[0]
    beta7 = _p(params, bn[7] + ".bias")
    P7 = maps[7]["s"][:, None] * maps[7]["Pp"]
    out = {"occ_out.0.weight": (P7 @ abar + beta7 * gbar)[None], "occ_out.0.bias": np.array([gbar])}
    A = np.outer(w, abar)                       # adjoint of P_7
    for L in range(7, -1, -1):
        m = maps[L]
        ds = (A * m["Pp"]).sum(1)
        out[bn[L] + ".weight"] = ds * m["r"]
        out[bn[L] + ".bias"] = w * gbar if L == 7 else np.zeros(256)
        dv = -0.5 * ds * m["gamma"] * m["r"] ** 3
        Ap = m["s"][:, None] * A + 2.0 * dv[:, None] * m["Q"]     # adjoint of P'_L
        out[lin[L] + ".bias"] = np.zeros(256)
        if L == 0:
            out[lin[L] + ".weight"] = Ap
            break
        Pprev = maps[L - 1]["s"][:, None] * maps[L - 1]["Pp"]
        W = m["W"]
        if L == 4:
            out[lin[L] + ".weight"] = np.concatenate([Ap, Ap @ Pprev.T], 1)
            A = W[:, 63:].T @ Ap
        else:
            out[lin[L] + ".weight"] = Ap @ Pprev.T
            A = W.T @ Ap
    return out
