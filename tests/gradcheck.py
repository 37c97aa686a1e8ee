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


def _report(line):
    """One JSON line per check into $PCNERF_PARITY_REPORT (the GPU run's parity report), when set."""
    import json
    import os
    path = os.environ.get("PCNERF_PARITY_REPORT")
    if path:
        with open(path, "a") as fh:
            fh.write(json.dumps(line) + "\n")


def check_grads_elem(get, keys, g, prefix, case, rtol=1e-4, spread_k=1.5, floor_k=6.0, noise=1e-5):
    """Per-element gradient parity against a reference run ``g`` that also holds the SAME computation rerun under
    another summation order (``alt:`` keys: the reference at another torch thread count) and, where present, its
    float64 evaluation (``f64:`` keys, tests/golden/make_f64.py grads).
    * with f64 keys: entry i passes when |hip_i - f64_i| <= max(rtol |f64_i|, spread_k |ref_i - f64_i| + floor):
      this path is as close to the exact gradient as the reference's own float32 result is; where the reference
      was also run at another thread count (``alt:``), |ref_i - f64_i| is the larger of its two runs' distances
      (one run's distance is one draw of a heavy-tailed error: the fine network's gradients at small BatchNorm
      chunks follow fine samples that one float32 ulp moves), and the tensor's RMS error must also stay within
      spread_k x the noisier run's RMS distance;
    * without: |hip_i - ref_i| <= max(rtol |ref_i|, spread_k |ref_i - alt_i| + floor);
    floor = floor_k x the RMS over the tensor of that spread (one sample of the reference's rounding noise per entry;
    the floor carries its typical size -- 6 RMS: the split products' operands carry 22 bits, float32's 24, so this
    path's rounding noise can be ~4x the reference's own).  Weight matrices are compared on their stored entries and by norm; the
    mathematically-zero gradients only at noise level.  Returns {tensor: (max err/tol, max |err| / max |ref|)} and
    reports it."""
    bad, worst = [], {}
    nz = noise_level_grads()
    for k in keys:
        gr = np.asarray(get(k), dtype=np.float64)
        try:
            if k in nz:
                ref_scale = np.abs(g[prefix + nz[k]]).max()
                assert np.abs(gr).max() <= noise * ref_scale, (np.abs(gr).max(), ref_scale)
                continue
            sfx = "" if prefix + k in g else "@val"
            f64 = "f64:" + prefix + k + sfx in g
            # with f64 keys, the reference's OTHER float32 run (alt:, another thread count) is a second sample of
            # its distance from the exact gradient
            ref2 = None
            if prefix + k in g:
                ref = g[prefix + k].astype(np.float64).ravel()
                alt = g[("f64:" if f64 else "alt:") + prefix + k].astype(np.float64).ravel()
                if f64 and "alt:" + prefix + k in g:
                    ref2 = g["alt:" + prefix + k].astype(np.float64).ravel()
                hip = gr.ravel()
            else:
                idx = g[prefix + k + "@idx"]
                ref = g[prefix + k + "@val"].astype(np.float64)
                alt = g[("f64:" if f64 else "alt:") + prefix + k + "@val"].astype(np.float64)
                if f64 and "alt:" + prefix + k + "@val" in g:
                    ref2 = g["alt:" + prefix + k + "@val"].astype(np.float64)
                hip = gr.reshape(-1)[idx]
                nr, na = float(g[prefix + k + "@norm"]), float(g[("f64:" if f64 else "alt:") + prefix + k + "@norm"])
                nt = na if f64 else nr
                assert abs(np.linalg.norm(gr) - nt) <= rtol * nt + spread_k * abs(nr - na), \
                    ("norm", np.linalg.norm(gr), nr, na)
            spread = np.abs(ref - alt)
            if ref2 is not None:   # the larger of the reference's two distances from the exact gradient
                spread = np.maximum(spread, np.abs(ref2 - alt))
            if f64:   # the exact gradient is the target, the reference's own distance from it the envelope
                ref, alt = alt, ref
            floor = floor_k * np.sqrt(np.mean(spread ** 2))
            tol = np.maximum(rtol * np.abs(ref), spread_k * spread + floor)
            err = np.abs(hip - ref)
            if ref2 is not None:   # and as a whole: no noisier than the reference's noisier run (RMS over the tensor)
                rms_ref = max(np.sqrt(np.mean((alt - ref) ** 2)), np.sqrt(np.mean((ref2 - ref) ** 2)))
                assert np.sqrt(np.mean(err ** 2)) <= spread_k * rms_ref + rtol * np.sqrt(np.mean(ref ** 2)), \
                    ("rms", float(np.sqrt(np.mean(err ** 2))), float(rms_ref))
            ratio = err / np.maximum(tol, 1e-300)
            i = int(np.argmax(ratio))
            worst[k] = (float(ratio[i]), float(err.max() / max(np.abs(ref).max(), 1e-300)))
            assert ratio[i] <= 1.0, (f"entry {i}: hip {hip[i]:.9g} ref {ref[i]:.9g} alt {alt[i]:.9g} tol {tol[i]:.3g}; "
                                     f"{int((ratio > 1).sum())} of {ratio.size} entries over")
        except AssertionError as e:
            bad.append(prefix + k + ": " + " ".join(str(e).split())[:300])
    if worst:
        kw = max(worst, key=lambda x: worst[x][0])
        _report({"case": case, "prefix": prefix, "tensors": len(worst), "max_err_over_tol": worst[kw][0],
                 "worst_tensor": kw, "max_abs_err_over_tensor_max": max(v[1] for v in worst.values()),
                 "failed": len(bad)})
    assert not bad, "\n".join(bad)
    return worst
