"""CPU check of the partitioning behind the slot-parallel record sums (csrc/gs_backward.hip,
k_sum_records_slots + k_sum_records_join): instance slots are cut into 64-slot chunks, each chunk
sums its owners' records and writes an owner that lies inside it directly, leaves the parts of an
owner that spans chunks (head [1], whole chunks and tail [0]) with IN / OUT / WHOLE flags, and the
join adds the parts from the head chunk on.  This restates that index logic in Python on random
owner layouts (runs of 1 to 300 slots) with integer values, so every Gaussian's total must be exact.
The kernels themselves are checked against the oracle on the GPU (tests/test_gpu_parity.py)."""
import numpy as np

SR_IN, SR_OUT, SR_WHOLE = 1, 2, 4


def chunked_sums(owners, vals):
    I = len(owners)
    nch = (I + 63) // 64
    out, part, flags = {}, np.zeros((nch, 2), dtype=np.int64), np.zeros(nch, dtype=np.int64)
    for c in range(nch):
        k0 = 64 * c
        nv = min(64, I - k0)
        gid, v = owners[k0:k0 + nv], vals[k0:k0 + nv]
        before = owners[k0 - 1] if k0 > 0 else -2
        after = owners[k0 + 64] if k0 + 64 < I else -2
        gf, gl = gid[0], gid[nv - 1]
        inn, out_ = before == gf, after == gl
        seg = np.zeros(nv, dtype=np.int64)  # segmented inclusive scan over the chunk
        for lane in range(nv):
            seg[lane] = v[lane] + (seg[lane - 1] if lane > 0 and gid[lane - 1] == gid[lane] else 0)
        for lane in range(nv):
            nxt = gid[lane + 1] if lane + 1 < nv else -3
            if nxt == gid[lane]:
                continue
            first_seg, last_seg = gid[lane] == gf, lane + 1 == nv
            if (first_seg and inn) or (last_seg and out_):
                part[c, 0 if (first_seg and inn) else 1] = seg[lane]
            else:
                assert gid[lane] not in out
                out[gid[lane]] = seg[lane]
        flags[c] = (SR_IN if inn else 0) | (SR_OUT if out_ else 0) | (SR_WHOLE if gf == gl else 0)
    for c in range(nch):  # the join
        f = flags[c]
        if not (f & SR_IN) or ((f & SR_WHOLE) and (f & SR_OUT)):
            continue
        h = c - 1
        while (flags[h] & SR_WHOLE) and (flags[h] & SR_IN):
            h -= 1
        g = owners[64 * c]
        assert g not in out
        out[g] = part[h, 1] + sum(part[j, 0] for j in range(h + 1, c + 1))
    return out


def test_chunked_record_sums_equal_per_owner_totals():
    rng = np.random.default_rng(0)
    for _ in range(200):
        V = int(rng.integers(1, 60))
        counts = rng.integers(1, rng.choice([3, 70, 300]), size=V)
        owners = np.repeat(rng.permutation(10 * V)[:V], counts)
        vals = rng.integers(-5, 6, size=len(owners))
        ref = {}
        for o, x in zip(owners, vals):
            ref[o] = ref.get(o, 0) + x
        assert chunked_sums(owners, vals) == ref
