"""Host check of the identity behind the attention kernels' packed-pair dropout (csrc/common.h
``drop_pair``): with both sides offset by 0x8000, the keep test ``half >= thr16`` (unsigned) is the
sign of a saturating signed 16-bit subtract, so ``v_pk_sub_i16 ... clamp`` followed by an
arithmetic shift by 15 gives an all-ones mask exactly for the dropped halves.  Exhaustive over the
16-bit half values for a spread of thresholds (0 and 65535 included)."""
import numpy as np


def _mask(half, thr):
    hs = (half ^ 0x8000).astype(np.uint16).view(np.int16).astype(np.int32)
    ts = np.int32(np.uint16(thr ^ 0x8000).view(np.int16))
    d = np.clip(hs - ts, -32768, 32767)  # v_pk_sub_i16 with clamp
    return (d >> 15) & 0xFFFF  # v_pk_ashrrev_i16 by 15: 0xFFFF where negative


def test_signed_offset_compare_equals_unsigned_keep_test():
    half = np.arange(65536, dtype=np.int64)
    for thr in [0, 1, 2, 6554, 13107, 32767, 32768, 32769, 58982, 65534, 65535]:
        dropped = _mask(half, thr) == 0xFFFF
        kept = _mask(half, thr) == 0
        assert np.array_equal(dropped, half < thr), thr
        assert np.array_equal(kept, half >= thr), thr


def test_pair_mask_zeroes_exactly_the_dropped_bf16_half():
    rng = np.random.default_rng(0)
    h = rng.integers(0, 2 ** 32, 4096, dtype=np.uint64).astype(np.uint32)
    pk = rng.integers(0, 2 ** 32, 4096, dtype=np.uint64).astype(np.uint32)
    thr = 6554  # p = 0.1
    lo, hi = h & 0xFFFF, h >> 16
    msk = _mask(lo.astype(np.int64), thr) | (_mask(hi.astype(np.int64), thr) << 16)
    out = pk & ~msk.astype(np.uint32)
    keep_lo, keep_hi = lo >= thr, hi >= thr
    assert np.array_equal(out & 0xFFFF, np.where(keep_lo, pk & 0xFFFF, 0))
    assert np.array_equal(out >> 16, np.where(keep_hi, pk >> 16, 0))
