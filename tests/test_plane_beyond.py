"""The shadow-ray plane skip (rtx_hip.hip plane_cand): for num, den of equal sign, an exact
|den| * tmax - |num| < 0 must imply RN(num / den) >= tmax, i.e. the reference's plane test
`t >= min && t < max` (Utils.h:82-104) fails and the division can be skipped.  The kernel
reads that sign off one fma; here the exact value comes from float64, where |den| * tmax
(24 x 24 bits) is exact and the subtraction keeps its sign."""
import numpy as np


def _cases(rng, n):
    den = rng.uniform(1e-3, 2.0, n).astype(np.float32) * rng.choice([-1, 1], n).astype(np.float32)
    tmax = rng.uniform(1e-3, 1e3, n).astype(np.float32)
    # num within a few ulps of den * tmax: the near-tie cases the skip must not misjudge
    near = (den * tmax).astype(np.float32).view(np.int32) + rng.integers(-4, 5, n).astype(np.int32)
    num = near.view(np.float32)
    return num, den, tmax


def test_beyond_implies_no_hit():
    rng = np.random.default_rng(7)
    for _ in range(4):
        num, den, tmax = _cases(rng, 1_000_000)
        same = np.signbit(num) == np.signbit(den)
        exact = np.abs(den).astype(np.float64) * tmax.astype(np.float64) - np.abs(num).astype(np.float64)
        beyond = same & (exact < 0)
        with np.errstate(all="ignore"):
            t = num / den   # float32 / float32: IEEE RN
        assert beyond.any()
        assert not np.any(beyond & (t < tmax)), "skip would drop a plane hit"
        # and the skip is tight: a same-sign lane not beyond can still be a hit
        assert np.any(same & ~beyond & (t < tmax))
