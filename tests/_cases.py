"""Shared test inputs (no tests here)."""
import numpy as np


def lambda_family(seed=3):
    """(H + lambda diag H) over alignFrames360's lambda schedule (1, then /5 per accepted update, :4589, :4718)
    for near-singular float Hessians (one direction almost unobserved, as on a textureless or planar level)."""
    rng = np.random.default_rng(seed)
    out = []
    for trial in range(40):
        A = rng.normal(size=(200, 6))
        A[:, 5] = A[:, 0] * rng.normal() + A[:, 1] * rng.normal() + rng.normal(size=200) * 10.0 ** rng.uniform(-6, -2)
        H = (A.T @ A).astype(np.float32)
        lam = 1.0
        for it in range(11):
            M = H.copy()
            for k in range(6):
                M[k, k] = np.float32(H[k, k] + np.float32(np.float32(lam) * H[k, k]))
            out.append((trial, it, M))
            lam /= 5.0
    return out
