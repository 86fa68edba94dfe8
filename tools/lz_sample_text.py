"""Config-2-like normalised text for tools/lz_model.c: the bench cohort's
depth model (tools/gen_cohort.cpp, restated in NumPy on 64 samples), step 4's
arithmetic in plain NumPy (normalize_mosdepth.py:419-499; a sample, not a
parity path), the row lines of write_normalized_output.

    python tools/lz_sample_text.py OUT.txt
"""
import sys

import numpy as np

rng = np.random.default_rng(5)
n, m, ncl = 64, 120000, 26
base = 25 + 30 * rng.random(m)
off = 0.16 * (rng.random((m, ncl)) - 0.5)
cl = rng.integers(0, ncl, n); scale = 0.6 + 0.8 * rng.random(n)
u1 = rng.random((n, m)); u2 = rng.random((n, m)); u3 = rng.random((n, m))
cnv = np.where(u3 < 0.02, np.where(u3 < 0.01, 0.5, 1.5), 1.0)
d = base[None] * (1 + off[:, cl].T) * scale[:, None] * cnv * (1 + 0.2 * (u1 + u2 - 1))
q = np.rint(d * 100) / 100
raw = q.mean(axis=1)
x = q / raw[:, None]
mu, var = x.mean(axis=0), x.var(axis=0, ddof=1)
ratio = 100 * var / mu
z = (x - mu) / np.sqrt(mu) / np.sqrt(np.median(ratio) / 100)
sel = np.nonzero(ratio > np.sort(ratio)[int(0.1 * m)])[0]
txt = "".join(f"S{i:05d}\t{raw[i]:.2f}\t" + "\t".join(f"{v:.2f}" for v in z[i, sel]) + "\n"
              for i in range(n)).encode()
open(sys.argv[1], 'wb').write(txt)
print(len(txt), len(sel), len(txt) / (n * len(sel)))
