"""Synthetic sources: counter-based splitmix64 streams, identical on the host
(numpy, for tests and the CPU baseline) and on the GPU (fw_generate_device, for benchmarks).

record i of stream `seed`:
  key = splitmix64(seed ^ 4i) mod num_keys      (uniform)   or   Zipf(s) rank via an inverse CDF
  val = (int32) splitmix64(seed ^ (4i + 1))
  ts  = ts_base + floor(i * 1000 / rate) - (splitmix64(seed ^ (4i + 2)) mod jitter)
Watermarks are punctuated: after each batch, wm = max(ts so far) - bound
(BoundedOutOfOrdernessTimestampExtractor.getCurrentWatermark, .../functions/timestamps/
BoundedOutOfOrdernessTimestampExtractor.java:70-76).
"""
import ctypes

import numpy as np

from . import _native as N

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(z):
    z = z.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        z += np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def zipf_cdf(num_keys, s):
    w = 1.0 / np.power(np.arange(1, num_keys + 1, dtype=np.float64), s)
    c = np.cumsum(w)
    c /= c[-1]
    c[-1] = 1.0
    return c


def generate_host(seed, first, n, num_keys, ts_base=0, rate=100_000_000, jitter=200, zipf_s=None, cdf=None):
    i = np.arange(first, first + n, dtype=np.uint64)
    s = np.uint64(seed)
    with np.errstate(over="ignore"):
        r0 = splitmix64(s ^ (np.uint64(4) * i))
        r1 = splitmix64(s ^ (np.uint64(4) * i + np.uint64(1)))
        r2 = splitmix64(s ^ (np.uint64(4) * i + np.uint64(2)))
    if zipf_s is not None or cdf is not None:
        if cdf is None:
            cdf = zipf_cdf(num_keys, zipf_s)
        u = (r0 >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
        keys = np.minimum(np.searchsorted(cdf, u, side="right"), num_keys - 1).astype(np.int64)
    else:
        keys = (r0 % np.uint64(num_keys)).astype(np.int64)
    vals = (r1 & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32).astype(np.int64)
    ts = np.int64(ts_base) + ((i * np.uint64(1000)) // np.uint64(rate)).astype(np.int64)
    if jitter > 0:
        ts = ts - (r2 % np.uint64(jitter)).astype(np.int64)
    return keys, ts, vals


def generate_device(seed, first, n, num_keys, ts_base=0, rate=100_000_000, jitter=200, cdf_dev=None, device=0,
                    out=None):
    """Generates on the GPU into torch int64 tensors; returns (keys, ts, vals, max_ts tensor)."""
    import torch
    dev = torch.device("cuda", device)
    if out is None:
        out = tuple(torch.empty(n, dtype=torch.int64, device=dev) for _ in range(3))
    keys, ts, vals = out
    mx = torch.full((1,), -(1 << 63), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    rc = N.lib().fw_generate_device(ctypes.c_uint64(seed), first, n, num_keys,
                                    cdf_dev.data_ptr() if cdf_dev is not None else None, ts_base, rate, jitter,
                                    keys.data_ptr(), ts.data_ptr(), vals.data_ptr(), mx.data_ptr(), stream)
    N.check(rc)
    return keys, ts, vals, mx
