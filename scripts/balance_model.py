"""Model of config 3's workgroup balance (CPU only): bytes per workgroup of
the spans kernel under the default deal (16-span blocks round robin over G
workgroups, then one span at a time: crc32c_dev.h wg_units) and under
HCRC_BALANCE's contiguous cut by weight (length + 64), for the bench's Zipf
mix (bench_extra.zipf_spans, 2 GiB) over several seeds.
  python scripts/balance_model.py [G]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_extra import BUCKETS, zipf_spans  # noqa: E402


def dealt(n, G):
    idx = np.arange(n)
    full = n // (16 * G) * 16
    return np.where(idx < full * G, (idx // 16) % G, (idx - full * G) % G)


def balanced(lens, G):
    w = lens.astype(np.float64) + 64.0
    excl = np.concatenate([[0.0], np.cumsum(w)[:-1]])
    T = w.sum()
    return np.minimum((excl * G / T).astype(np.int64), G - 1)


def main():
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    for seed in range(1, 6):
        rng = np.random.default_rng(seed)
        _, lens, _ = zipf_spans(rng, 2 << 30, BUCKETS)
        out = []
        for name, wg in (("dealt", dealt(lens.size, G)), ("balanced", balanced(lens, G))):
            s = np.bincount(wg, weights=lens.astype(np.float64), minlength=G)
            out.append(f"{name} max/mean {s.max() / s.mean():.3f} sd/mean {s.std() / s.mean():.4f}")
        print(f"seed {seed}: {lens.size} spans, {lens.size / G:.0f} per workgroup; " + "; ".join(out))


if __name__ == "__main__":
    main()
