"""Portable synthetic client state.

A counter-based integer hash (splitmix64 finaliser) that is restated
bit-for-bit in numpy (here) and in HIP (``fa_synth_fill_*`` in
csrc/fedagg.hip), so the GPU box regenerates the exact inputs the golden
digests were computed from without shipping hundreds of MB of fixtures.

Every float is produced with exactly-representable integer→float steps
followed by single correctly-rounded fp32 multiplies/adds (no FMA), so numpy
and the HIP kernel agree bit-for-bit.

Element value of client ``c`` (seed ``1000 + c``), key ``k``, flat index ``e``
inside the key's tensor, ``idx = (k << 36) | e``:

  realistic:   x = (mu + sigma * s(h(BASE_SEED, idx))) + (0.01*sigma) * s(h(seed, idx))
  adversarial: x = s(h(seed, idx)) * 2**(ex),  ex = (h(seed, idx) >> 8) % 41 - 20
  int64:       realistic  19*round + h(seed, idx) % 7
               adversarial (h % 2**26) - 2**25

with ``s(h) = ((h >> 40) - 2**23) * 2**-23`` in [-1, 1).
"""
from __future__ import annotations

import math

import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
GOLDEN = np.uint64(0x9E3779B97F4A7C15)
MUL_IDX = np.uint64(0xD1B54A32D192ED03)
MIX1 = np.uint64(0xBF58476D1CE4E5B9)
MIX2 = np.uint64(0x94D049BB133111EB)
BASE_SEED = 7
CLIENT_SEED0 = 1000
KEY_SHIFT = 36
ROUND = 5

MODE_REALISTIC = 0
MODE_ADVERSARIAL = 1


def hash64(seed: int, idx: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser of ``seed*GOLDEN + idx*MUL_IDX`` (mod 2**64)."""
    idx = np.asarray(idx, np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) * GOLDEN + idx * MUL_IDX
        z = (z ^ (z >> np.uint64(30))) * MIX1
        z = (z ^ (z >> np.uint64(27))) * MIX2
        z = z ^ (z >> np.uint64(31))
    return z


def sym_unit(h: np.ndarray) -> np.ndarray:
    """Top 24 bits of h → float32 in [-1, 1), exactly."""
    v = (h >> np.uint64(40)).astype(np.int64) - (1 << 23)
    return v.astype(np.float32) * np.float32(2.0 ** -23)


def key_params(name: str, shape, dtype: str):
    """(mu, sigma) for a state_dict key, by role (kaiming fan-out for convs)."""
    if dtype != "float32":
        return 0.0, 0.0
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "running_var":
        return 1.0, 0.1
    if leaf in ("running_mean", "bias"):
        return 0.0, 0.1
    if leaf == "weight" and len(shape) == 1:
        return 1.0, 0.1
    if len(shape) == 4:
        fan_out = shape[0] * shape[2] * shape[3]
        return 0.0, math.sqrt(2.0 / fan_out)
    if len(shape) == 2:
        return 0.0, 1.0 / math.sqrt(shape[1])
    return 0.0, 0.1


def key_consts(mu: float, sigma: float):
    """The three fp32 constants the generator uses (as the HIP side does)."""
    return np.float32(mu), np.float32(sigma), np.float32(np.float32(sigma) * np.float32(0.01))


def gen_f32(key_index: int, numel: int, client: int, mu: float, sigma: float,
            mode: int = MODE_REALISTIC) -> np.ndarray:
    idx = (np.uint64(key_index) << np.uint64(KEY_SHIFT)) | np.arange(numel, dtype=np.uint64)
    hc = hash64(CLIENT_SEED0 + client, idx)
    if mode == MODE_ADVERSARIAL:
        ex = ((hc >> np.uint64(8)) % np.uint64(41)).astype(np.int64) - 20
        scale = np.ldexp(np.float32(1.0), ex).astype(np.float32)
        return (sym_unit(hc) * scale).astype(np.float32)
    m, s, d = key_consts(mu, sigma)
    base = (m + (s * sym_unit(hash64(BASE_SEED, idx))).astype(np.float32)).astype(np.float32)
    return (base + (d * sym_unit(hc)).astype(np.float32)).astype(np.float32)


def gen_i64(key_index: int, numel: int, client: int, mode: int = MODE_REALISTIC) -> np.ndarray:
    idx = (np.uint64(key_index) << np.uint64(KEY_SHIFT)) | np.arange(numel, dtype=np.uint64)
    hc = hash64(CLIENT_SEED0 + client, idx)
    if mode == MODE_ADVERSARIAL:
        return (hc % np.uint64(1 << 26)).astype(np.int64) - (1 << 25)
    return (19 * ROUND + (hc % np.uint64(7)).astype(np.int64)).astype(np.int64)


def gen_key(key_index: int, name: str, shape, dtype: str, client: int,
            mode: int = MODE_REALISTIC) -> np.ndarray:
    numel = int(np.prod(shape)) if len(shape) else 1
    if dtype == "int64":
        return gen_i64(key_index, numel, client, mode).reshape(shape)
    mu, sigma = key_params(name, shape, dtype)
    return gen_f32(key_index, numel, client, mu, sigma, mode).reshape(shape)


def gen_state(manifest, client: int, mode: int = MODE_REALISTIC):
    """Ordered list of (key, ndarray) for one client, following a manifest."""
    return [(e["key"], gen_key(i, e["key"], tuple(e["shape"]), e["dtype"], client, mode))
            for i, e in enumerate(manifest["keys"])]
