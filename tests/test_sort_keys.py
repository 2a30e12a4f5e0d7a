"""Host checks of the sort kernel's packed-key encoding (csrc/dpg_sortb.h):
the narrow kernel sorts keys `01 | pid slot (7) | top min(32, 45 - pkbits)
priority bits | pk | position (9)` with float64 min / max, which is only valid if
every such key read as a float64 is a finite, positive, normal number whose
float order equals the unsigned order of its bits, and if the padding key
(+inf) sorts after all of them.  (The GPU parity tests cover the kernel.)"""
import numpy as np
import pytest

TAG = 1 << 61
PAD = 0x7FF0000000000000


def _pack(slot, prio, pk, pos, pkbits):
    ppb = min(32, 45 - int(pkbits))
    return (TAG | (slot << 54) | ((prio >> (32 - ppb)) << (9 + pkbits)) | (pk << 9) | pos)


@pytest.mark.parametrize("pkbits", [1, 12, 20, 24])
def test_packed_keys_float_order_is_bit_order(pkbits):
    rng = np.random.default_rng(pkbits)
    n = 200_000
    slot = rng.integers(0, 128, n, dtype=np.uint64)
    prio = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    pk = rng.integers(0, 1 << pkbits, n, dtype=np.uint64)
    pos = rng.integers(0, 512, n, dtype=np.uint64)
    keys = _pack(slot, prio, pk, pos, np.uint64(pkbits)).astype(np.uint64)
    # extremes of every field
    ext = [_pack(s, p, k, q, pkbits) for s in (0, 127) for p in (0, (1 << 32) - 1)
           for k in (0, (1 << pkbits) - 1) for q in (0, 511)]
    keys = np.concatenate([keys, np.array(ext, dtype=np.uint64)])
    assert int(keys.max()) < (1 << 62) and int(keys.min()) >= TAG
    f = keys.view(np.float64)
    assert np.all(np.isfinite(f)) and np.all(f > 0)
    assert np.all(np.abs(f) >= np.finfo(np.float64).tiny)       # normal, not denormal
    order_bits = np.argsort(keys, kind="stable")
    order_float = np.argsort(f, kind="stable")
    assert np.array_equal(keys[order_bits], keys[order_float])
    pad = np.array([PAD], dtype=np.uint64).view(np.float64)[0]
    assert np.isinf(pad) and np.all(f < pad)
