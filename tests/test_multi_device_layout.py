"""The multi-device layout (include/vs.h vs_multi_*, csrc/vs_multi.hip) restated on the CPU: rows are
dealt in chunks of 2^16 consecutive ids (chunk j on shard j mod G); a shard's local row l has
global id ((l >> 16) * G + g) << 16 | (l & 0xFFFF).  Checked here with the oracle as the index: the
dealing is balanced and order-preserving, ids round-trip, and merging the shards' exact top-k
lists (score, then lower GLOBAL id) equals one exact search over all rows -- including exact ties
split across shards."""
import numpy as np

from oracle import oracle as O

BITS = 16


def deal(G, r0, n):
    """Per shard, the (batch offset, count) pieces of global rows [r0, r0 + n) -- vs_multi's split_rows."""
    out = [[] for _ in range(G)]
    i = 0
    while i < n:
        gid = r0 + i
        chunk = gid >> BITS
        m = min(n - i, ((chunk + 1) << BITS) - gid)
        out[chunk % G].append((i, m))
        i += m
    return out


def to_global(l, G, g):
    l = np.asarray(l, dtype=np.int64)
    return np.where(l < 0, -1, ((((l >> BITS) * G) + g) << BITS) | (l & ((1 << BITS) - 1)))


def test_dealing_is_balanced_and_ids_round_trip():
    G, N = 3, 10 * (1 << BITS) + 123
    owner = np.empty(N, dtype=np.int64)
    local = np.empty(N, dtype=np.int64)
    counts = [0] * G
    for r0, n in ((0, 1), (1, 70_000), (70_001, 5), (70_006, N - 70_006)):  # incremental + bulk adds
        for g, pieces in enumerate(deal(G, r0, n)):
            for off, m in pieces:
                owner[r0 + off:r0 + off + m] = g
                local[r0 + off:r0 + off + m] = np.arange(counts[g], counts[g] + m)
                counts[g] += m
    assert max(counts) - min(counts) <= 1 << BITS
    for g in range(G):
        sel = np.flatnonzero(owner == g)
        np.testing.assert_array_equal(to_global(local[sel], G, g), sel)  # order-preserving, exact inverse


def test_merged_shard_lists_equal_one_search_with_ties_across_shards():
    G, d, k = 2, 16, 30
    N = 3 * (1 << BITS) // 8
    rng = np.random.default_rng(1)
    x = rng.standard_normal((N, d)).astype(np.float32)
    x[N // 2:N // 2 + 40] = x[7]  # exact duplicates of row 7 (ties -> lower global id)
    q = np.concatenate([x[7:8], rng.standard_normal((5, d)).astype(np.float32)])
    # deal as if these rows were global ids [2^16 - N/2, 2^16 + N/2): the duplicates straddle a chunk
    base = (1 << BITS) - N // 2
    S_parts, I_parts = [], []
    for g, pieces in enumerate(deal(G, base, N)):
        rows = np.concatenate([np.arange(off, off + m) for off, m in pieces]) if pieces else np.zeros(0, np.int64)
        S, I = O.knn_exact(x[rows], q, k, "ip")
        # the shard's local ids -> global ids (its local numbering starts after the chunks before base)
        first_local = sum(min(1 << BITS, base - (c << BITS)) for c in range((base >> BITS) + 1) if c % G == g)
        gl = to_global(np.where(I >= 0, I + first_local, -1), G, g)
        S_parts.append(S)
        I_parts.append(gl - base)  # back to row numbers of x for the comparison
    Sm, Im = O.merge_topk(np.stack(S_parts), np.stack(I_parts), k, "ip")
    Se, Ie = O.knn_exact(x, q, k, "ip")
    np.testing.assert_array_equal(Im, Ie)
    np.testing.assert_array_equal(Sm, Se)
