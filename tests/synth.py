"""Seeded synthetic metrology data — test infrastructure.

Counter-based (splitmix64 keyed by seed, stream, index) so any sub-block can be regenerated
independently.  Model (src/Modulation.jl:57-64, tex/GPPupilDemodulation.tex:134-142):
    d_i = p_i · (c + a · exp(j b sin(ω t_i + ϕ))) + σ · CN(0,1)
with p_i = exp(j Φ_i) the fibre-coupler (FC) phasor, Φ a Gaussian random walk shared by each
group of 4 diodes.
"""
from __future__ import annotations

import numpy as np

M_2PI = 6.283185  # src/Modulation.jl:11

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
    z = x
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
    return z ^ (z >> np.uint64(31))


def uniform(seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    """U[0,1) doubles keyed by (seed, stream, idx)."""
    with np.errstate(over="ignore"):
        key = _splitmix(np.uint64(seed) * np.uint64(0x100000001B3) ^ np.uint64(stream))
        z = _splitmix(np.asarray(idx, dtype=np.uint64) ^ key)
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def normal(seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    u1 = uniform(seed, 2 * stream, idx)
    u2 = uniform(seed, 2 * stream + 1, idx)
    return np.sqrt(-2.0 * np.log1p(-u1)) * np.cos(2 * np.pi * u2)


def make_batch(n_samples: int, n_pixels: int, seed: int = 1, t0: float = 0.0, dt: float = 0.002,
               sigma: float = 0.1, offsets: bool = False, group: int = 4,
               b_range=(0.3, 2.5), omega: float = M_2PI):
    """Returns dict(t, d (P×N), fc (G×N), fc_of_pixel (P,), truth dict)."""
    N, P = n_samples, n_pixels
    G = (P + group - 1) // group
    t = t0 + np.arange(N, dtype=np.float64) * dt
    pix = np.arange(P, dtype=np.uint64)
    b = b_range[0] + (b_range[1] - b_range[0]) * uniform(seed, 1, pix)
    phi = -np.pi + 2 * np.pi * uniform(seed, 2, pix)
    amp = 0.5 + uniform(seed, 3, pix)
    arga = -np.pi + 2 * np.pi * uniform(seed, 4, pix)
    a = amp * np.exp(1j * arga)
    if offsets:
        c = 0.1 * (normal(seed, 5, pix) + 1j * normal(seed, 6, pix)) / np.sqrt(2)
    else:
        c = np.zeros(P, dtype=np.complex128)
    fc = np.empty((G, N), dtype=np.complex128)
    ii = np.arange(N, dtype=np.uint64)
    for g in range(G):
        steps = 1e-3 * normal(seed, 100 + g, ii)
        Phi = np.cumsum(steps) + 2 * np.pi * uniform(seed, 7, np.array([g], dtype=np.uint64))[0]
        fc[g] = 1.3 * np.exp(1j * Phi)
    fc_of_pixel = (np.arange(P) // group).astype(np.int32)
    d = np.empty((P, N), dtype=np.complex128)
    for k in range(P):
        p = fc[fc_of_pixel[k]] / np.abs(fc[fc_of_pixel[k]])
        model = c[k] + a[k] * np.exp(1j * b[k] * np.sin(omega * t + phi[k]))
        noise = (normal(seed, 1000 + 2 * k, ii) + 1j * normal(seed, 1001 + 2 * k, ii)) / np.sqrt(2)
        d[k] = p * model + sigma * noise
    return dict(t=t, d=d, fc=fc, fc_of_pixel=fc_of_pixel,
                truth=dict(a=a, b=b, phi=phi, c=c))


def wrap(x):
    return (np.asarray(x) + np.pi) % (2 * np.pi) - np.pi
