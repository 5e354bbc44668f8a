"""CPU checks of the arithmetic lemmas the fast paths rest on.

N32: floor(fl32(x * RU32(100/M))) == floor(100 x / M) whenever 300 x + M < 2^24.
F64: floor(fl64(x * RU64(100/M))) == floor(100 x / M) whenever x, M <= 2^44.
Both are proven in DESIGN.md; here they are checked exhaustively on a sub-domain and by
random sampling over the whole domain (tools/check_div_lemma.c runs the full exhaustive
M <= 60000 sweep in ~10 s)."""
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def ru32(M):
    r = (np.float64(100.0) / M.astype(np.float64)).astype(np.float32)
    low = np.fma(r.astype(np.float64), M.astype(np.float64), -100.0) < 0 \
        if hasattr(np, "fma") else (r.astype(np.float64) * M < 100.0)
    return np.where(low, np.nextafter(r, np.float32(np.inf)), r)


def ru64(M):
    r = 100.0 / M.astype(np.float64)
    # exact sign of r*M - 100 via the two-product of r and M
    prod = r * M
    err = np.array([float(np.longdouble(a) * np.longdouble(b) - np.longdouble(c))
                    for a, b, c in zip(r, M.astype(np.float64), prod)])
    below = (prod < 100.0) | ((prod == 100.0) & (err < 0))
    return np.where(below, np.nextafter(r, np.inf), r)


def test_n32_lemma_exhaustive_small_domain():
    for M in range(1, 3001):
        x = np.arange(0, min(M, (1 << 24) // 300) + 1, dtype=np.uint64)
        r = ru32(np.array([M], dtype=np.uint64))[0]
        q = (x.astype(np.float32) * r).astype(np.uint32)
        want = (x * 100) // M
        assert np.array_equal(q, want), M


def test_n32_lemma_random_whole_domain():
    rng = np.random.default_rng(0)
    M = rng.integers(1, 1 << 24, size=200_000).astype(np.uint64)
    xmax = ((1 << 24) - 1 - M) // 300
    x = (rng.random(M.size) * (xmax + 1)).astype(np.uint64)
    x = np.where(rng.random(M.size) < 0.5, xmax, x)  # the boundary
    q = (x.astype(np.float32) * ru32(M)).astype(np.uint64)
    assert np.array_equal(q, (x * 100) // M)


def test_f64_lemma_random():
    rng = np.random.default_rng(1)
    M = rng.integers(1, 1 << 44, size=20_000, dtype=np.int64).astype(np.uint64)
    x = (rng.random(M.size) * (M.astype(np.float64) + 1)).astype(np.uint64)
    x = np.minimum(x, M)
    r = ru64(M)
    q = np.floor(x.astype(np.float64) * r).astype(np.uint64)
    want = np.array([(int(a) * 100) // int(b) for a, b in zip(x, M)], dtype=np.uint64)
    assert np.array_equal(q, want)


def test_c_checker_builds_and_passes_random():
    exe = "/tmp/yoda_check_div_lemma"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe,
                    os.path.join(REPO, "tools", "check_div_lemma.c"), "-lm"], check=True)
    out = subprocess.run([exe, "r", "20000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    out = subprocess.run([exe, "4000", "4000"], capture_output=True, text=True)
    assert out.returncode == 0 and "0 mismatches" in out.stdout, out.stdout
