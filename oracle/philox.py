"""TEST INFRASTRUCTURE ONLY -- Philox4x32-10 keyed draw contract, numpy form.

The reference draws from the unseeded global NumPy RandomState
(utils/graph.py:218, :328, :380, :420, :457; utils/batch_loader.py:40-41;
utils/null_model.py:23).  Bit-exact parity is only defined under an injected
keyed RNG.  The contract, shared by this module, the C
oracle (oracle/tempme_oracle.c) and the HIP kernels (tempme_amd/csrc/rng.h):

    key     = (seed & 0xffffffff, seed >> 32)
    counter = (event, (split << 16) | (side << 8) | stage, row, j >> 2)
    u32     = philox4x32_10(counter, key)[j & 3]
    draw(high) = (u32 * high) >> 32            # value in [0, high)

``row`` is the row index inside the event (hop-h row, step-2 slot, walk) and
``j`` the draw index inside the row (the reference's ``randint(..., size)``
vector position).  The vector of draws is then sorted (np.sort) exactly as the
reference does.
"""
import numpy as np

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF

# splits
SPLIT_TRAIN, SPLIT_TEST, SPLIT_NULL = 0, 1, 2
# sides
SIDE_NONE, SIDE_SRC, SIDE_TGT, SIDE_BGD = 0, 1, 2, 3
# stages (hop h of find_k_hop uses stage h, 1 <= h <= 15)
STAGE_STEP2, STAGE_STEP3, STAGE_NEG, STAGE_PERM = 16, 17, 32, 48


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 (Salmon et al., SC'11).  uint64 arrays in/out."""
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint64) & MASK for x in (c0, c1, c2, c3))
    k0 = np.asarray(k0, dtype=np.uint64) & MASK
    k1 = np.asarray(k1, dtype=np.uint64) & MASK
    for r in range(10):
        if r:
            k0 = (k0 + W0) & MASK
            k1 = (k1 + W1) & MASK
        p0 = np.uint64(M0) * c0
        p1 = np.uint64(M1) * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & np.uint64(MASK)
        hi1, lo1 = p1 >> np.uint64(32), p1 & np.uint64(MASK)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
    return c0, c1, c2, c3


def tag(split, side, stage):
    return (split << 16) | (side << 8) | stage


def draw_u32(seed, split, side, stage, event, row, j):
    event = np.asarray(event, dtype=np.uint64)
    row = np.asarray(row, dtype=np.uint64)
    j = np.asarray(j, dtype=np.uint64)
    event, row, j = np.broadcast_arrays(event, row, j)
    t = np.full(event.shape, tag(split, side, stage), dtype=np.uint64)
    out = philox4x32_10(event, t, row, j >> np.uint64(2), seed & MASK, (seed >> 32) & MASK)
    words = np.stack(out, axis=-1)
    return np.take_along_axis(words, (j & np.uint64(3)).astype(np.int64)[..., None], axis=-1)[..., 0]


def draw(seed, split, side, stage, event, row, j, high):
    """Keyed replacement for ``np.random.randint(0, high)`` (per element)."""
    u = draw_u32(seed, split, side, stage, event, row, j)
    return ((u * np.asarray(high, dtype=np.uint64)) >> np.uint64(32)).astype(np.int64)


def keyed_permutation(n, seed, split=SPLIT_NULL):
    """Keyed replacement for ``np.random.permutation(n)`` (utils/null_model.py:23):
    stable argsort of one Philox word per position."""
    keys = draw_u32(seed, split, SIDE_NONE, STAGE_PERM, np.arange(n), 0, 0)
    return np.argsort(keys, kind="stable").astype(np.int64)
