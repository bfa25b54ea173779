"""Counter-based synthetic client updates (SURVEY.md §8(d) "Input generation").

Every value is a pure function of ``(seed, stream, index)``, so the same bits
are produced by this numpy restatement, by the C oracle
(``oracle/fedagg_oracle.c: flame_oracle_synth``) and by the HIP generator
(``flame_amd/csrc/fedagg.hip: synth_kernel``).  That lets 100 GB of client
updates be generated in HBM for device-resident timing and regenerated
bit-identically on the host for sampled parity checks.

Generator (all integer arithmetic wraps mod 2**64):

    mix64(z)  = splitmix64 finaliser
    ck        = mix64(seed * GAMMA  ^  (stream + 1) * STREAM_MUL)
    h         = mix64(ck + index * GAMMA)
    s         = (h & 0xffff) + (h>>16 & 0xffff) + (h>>32 & 0xffff) + (h>>48) - 131070
    value_f32 = float32(s) * scale_f32          (one IEEE RNE multiply)

``s`` is an Irwin-Hall(4) sum, approximately normal; ``float32(s)`` is exact
(|s| < 2**24) so the single multiply is the only rounding.  bf16 / f16 data
are ``value_f32`` rounded to nearest-even.
"""
from __future__ import annotations

import math

import numpy as np

GAMMA = 0x9E3779B97F4A7C15
STREAM_MUL = 0xD1B54A32D192ED03
M1 = 0xBF58476D1CE4E5B9
M2 = 0x94D049BB133111EB
MASK64 = (1 << 64) - 1
# standard deviation of a sum of four discrete uniforms on {0..65535}
IH4_STD = math.sqrt((65536.0 ** 2 - 1.0) / 3.0)


def scale_for_sigma(sigma: float) -> np.float32:
    """fp32 multiplier that gives the generator standard deviation ``sigma``."""
    return np.float32(sigma / IH4_STD)


def _mix64_int(z: int) -> int:
    z &= MASK64
    z = ((z ^ (z >> 30)) * M1) & MASK64
    z = ((z ^ (z >> 27)) * M2) & MASK64
    return z ^ (z >> 31)


def stream_key(seed: int, stream: int) -> int:
    return _mix64_int(((seed * GAMMA) & MASK64) ^ (((stream + 1) * STREAM_MUL) & MASK64))


def _mix64_np(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * np.uint64(M1)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(M2)
    return z ^ (z >> np.uint64(31))


def synth_f32(seed: int, stream: int, index, sigma: float) -> np.ndarray:
    """fp32 values for element indices ``index`` (int array or range length)."""
    if np.isscalar(index):
        idx = np.arange(int(index), dtype=np.uint64)
    else:
        idx = np.asarray(index, dtype=np.uint64)
    ck = np.uint64(stream_key(seed, stream))
    with np.errstate(over="ignore"):
        h = _mix64_np(ck + idx * np.uint64(GAMMA))
    m = np.uint64(0xFFFF)
    s = ((h & m) + ((h >> np.uint64(16)) & m) + ((h >> np.uint64(32)) & m)
         + (h >> np.uint64(48))).astype(np.int64) - 131070
    return s.astype(np.float32) * scale_for_sigma(sigma)


def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even fp32 -> bf16, returned as uint16 bit patterns."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) >> np.uint64(16))
    out = r.astype(np.uint16)
    nan = np.isnan(x)
    if nan.any():
        out[nan] = ((u[nan] >> np.uint64(16)) | np.uint64(0x40)).astype(np.uint16)
    return out


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << np.uint32(16)).view(np.float32)


def counts(seed: int, n: int, lo: int = 1, hi: int = 1000) -> np.ndarray:
    """Per-client dataset sizes ~ U{lo..hi} (host metadata, not device data)."""
    out = np.empty(n, dtype=np.int64)
    for i in range(n):
        out[i] = lo + _mix64_int(stream_key(seed ^ 0xC0FFEE, i)) % (hi - lo + 1)
    return out
