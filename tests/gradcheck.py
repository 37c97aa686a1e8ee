"""Shared gradient comparison for the training-gradient tests (oracle vs reference goldens, HIP vs both)."""
import numpy as np

from oracle import ref_cpu as O


def noise_level_grads():
    """Gradients that are mathematically zero: the bias of every Linear that feeds a BatchNorm (BN removes the
    mean) and the shift of every BN followed by Linear->BN (its gradient is W^T sum(dL/dh) = 0).  Their values
    are pure rounding noise, so they are checked to be at noise level against the BN scale gradient."""
    out = {}
    for i, (lin, bn) in enumerate(zip(O.LIN, O.BN)):
        out[lin + ".bias"] = bn + ".weight"
        if i < 7:
            out[bn + ".bias"] = bn + ".weight"
    return out


def check_grads(get, keys, g, prefix, rtol, noise=1e-5):
    """Golden gradients: small tensors in full, weight matrices by norm + 2048 fixed entries."""
    bad = []
    nz = noise_level_grads()
    for k in keys:
        gr = np.asarray(get(k), dtype=np.float64)
        try:
            if k in nz:
                ref_scale = np.abs(g[prefix + nz[k]]).max()
                assert np.abs(gr).max() <= noise * ref_scale, (np.abs(gr).max(), ref_scale)
                assert np.abs(g[prefix + k]).max() <= noise * ref_scale
            elif prefix + k in g:
                ref = g[prefix + k]
                np.testing.assert_allclose(gr, ref, rtol=rtol, atol=rtol * np.abs(ref).max(), err_msg=k)
            else:
                idx = g[prefix + k + "@idx"]
                ref = g[prefix + k + "@val"]
                np.testing.assert_allclose(gr.reshape(-1)[idx], ref, rtol=rtol, atol=rtol * np.abs(ref).max(),
                                           err_msg=k)
                np.testing.assert_allclose(np.linalg.norm(gr), g[prefix + k + "@norm"], rtol=rtol)
        except AssertionError as e:
            bad.append(prefix + k + ": " + " ".join(str(e).split())[:300])
    assert not bad, "\n".join(bad)
