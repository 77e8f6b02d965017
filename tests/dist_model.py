"""CPU model of the coset-sharded FRI commit (test infrastructure).

Mirrors run_commit_sharded (stark-prover_amd/csrc/fri_sharded.hip) step for step
with the same index math, using the C oracle for per-block work and
torch.distributed (gloo) for the exchanges:

  layer 0   rank r: P mod (x^M - s^M), s = offset*w_n^r, size-M LDE on s*<w_M>
            -> evals[r + G*m];  all-to-all of M/G chunks;  block[G*t + r] = recv[r][t]
  layer k   block-local Merkle tree; all-gather block roots; reorder by
            block_of; top log2(G) levels + channel (identical on every rank)
  fold      ranks holding blocks b and b + G/2 swap half-blocks; A keeps the
            first half of the outputs, B the second; block_of <- 2b / 2b'+1
  switch    below 2^shard_min_log: all-gather the layer, finish locally.
  degree    next_fri_polynomial (fri_commit.rs:32-50) sharded like k_coef:
            rank r folds coefficients [r*S_k, (r+1)*S_k) of poly_k; its
            maxima (nonzero c'_j, even part, odd part) and its first
            coefficient ride with the block root in the per-layer all-gather;
            deg_k and the final value follow from the G records; the chunks
            are all-gathered once at the switch.
"""
import ctypes
import hashlib

import numpy as np
import torch
import torch.distributed as dist

import fri_oracle as fo

P = fo.P


def _lde(lib, coeffs, log_m, offset):
    c = np.ascontiguousarray(np.asarray(coeffs, dtype=np.uint64))
    out = np.zeros(1 << log_m, dtype=np.uint64)
    lib.orc_lde(c.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), c.size, log_m, offset, 5, P,
                out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    return out


def _tree_root(lib, vals):
    v = np.ascontiguousarray(np.asarray(vals, dtype=np.uint64))
    cnt = lib.orc_merkle_nodes_count(v.size)
    buf = ctypes.create_string_buffer(32 * cnt)
    lib.orc_merkle_build(v.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), v.size, buf)
    return buf.raw[32 * (cnt - 1):]


def _allgather_bytes(b, world):
    t = torch.frombuffer(bytearray(b), dtype=torch.uint8)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    return [bytes(o.numpy()) for o in outs]


def _allgather_u64(a, world):
    t = torch.from_numpy(np.ascontiguousarray(a.astype(np.int64)))
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    return [o.numpy().astype(np.uint64) for o in outs]


def _allgather_records(rec, world):
    """(root bytes, m0, m1, m2, c0) of every rank, in rank order."""
    root, m = rec[0], np.array(rec[1:], dtype=np.int64)
    roots = _allgather_bytes(root, world)
    t = torch.from_numpy(m)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    return [(roots[r],) + tuple(int(x) for x in outs[r].numpy()) for r in range(world)]


def _rounds_bound(d, log_n):                          # fri_host.hpp rounds_bound
    return 0 if d <= 1 else min((d - 1).bit_length(), log_n)


def _coef_slice(k, prev, d, deg_prev, beta, lo, hi):
    """One rank's share of the coefficient task of layer k (k_coef,
    fri_layer.hip coef_task): k == 0 scans input indices [lo, hi) ∩ [0, d);
    k >= 1 folds c'_j = c_2j + beta*c_2j+1 for j in [lo, hi) ∩ [0, nlen).
    prev maps a global index of poly_{k-1} (the input at k == 1) to its value.
    Returns (chunk {j: c'_j}, m0, m1, m2) with global indices."""
    m0 = m1 = m2 = -1
    out = {}
    if k == 0:
        for j in range(lo, min(hi, d)):
            c = prev(j)
            if c:
                m0 = j
            if c >= P:
                m1 = 0
        return out, m0, m1, m2
    ln = deg_prev + 1
    nlen = (ln + 1) // 2
    for j in range(lo, min(hi, nlen)):
        e = prev(2 * j)
        o = prev(2 * j + 1) if 2 * j + 1 < ln else 0
        v = (e + beta * o) % P
        out[j] = v
        if v:
            m0 = j
        if e:
            m1 = j
        if o:
            m2 = j
    return out, m0, m1, m2


def sharded_commit(coeffs, log_n, rank, world, offset=fo.GEN, shard_min_log=8):
    lib = fo.load_c_oracle()
    G = world
    logG = G.bit_length() - 1
    n = 1 << log_n
    M = n // G
    d = len(coeffs)
    ch = fo.Channel()
    # ---- layer 0: coset slice + all-to-all + transpose -------------------
    wn = fo.fe_pow(5, (P - 1) // n, P)
    s = fo.fe_mul(offset, fo.fe_pow(wn, rank, P), P)
    c = fo.fe_pow(s, M, P)
    red = [0] * M
    for j in range(M):
        acc, t = 0, (d - 1 - j) // M if d > j else -1
        while t >= 0:
            acc = (acc * c + coeffs[j + t * M]) % P
            t -= 1
        red[j] = acc
    slice_ = _lde(lib, red, log_n - logG, s)                     # evals[rank + G*m]
    send = torch.from_numpy(slice_.astype(np.int64))
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send)
    per = M // G
    r_ = recv.numpy().astype(np.uint64).reshape(G, per)
    block = r_.T.reshape(-1).copy()                              # block[G*t + r] = recv[r][t]
    block_of = list(range(G))
    # coefficient chunks (plan_layout): G * S_0 >= d and S_k >= 1 up to the
    # last sharded layer
    rmax = _rounds_bound(d, log_n)
    k_sw = 0
    while k_sw < rmax and log_n - k_sw - 1 >= shard_min_log and log_n - k_sw - 1 - logG >= 1:
        k_sw += 1
    cs0 = max((-(-d // G) - 1).bit_length() if d > G else 0, k_sw)
    chunk = None                                                 # this rank's chunk of poly_{k}, {global j: value}
    deg, beta = -1, 0
    roots, betas = [], []
    k = 0
    inv2 = fo.fe_inverse(2, P)
    while True:
        Lk = log_n - k
        B = 1 << (Lk - logG)
        Sk = 1 << (cs0 - k)
        prev = (lambda j: coeffs[j] if j < d else 0) if k <= 1 else (lambda j, ch_=chunk: ch_[j])
        chunk, m0, m1, m2 = _coef_slice(k, prev, d, deg, beta, rank * Sk, (rank + 1) * Sk)
        c0 = (coeffs[0] if d else 0) if k == 0 else chunk.get(rank * Sk, 0)
        recs = _allgather_records((_tree_root(lib, block), m0, m1, m2, c0), G)
        ordered = [None] * G
        for r in range(G):
            ordered[block_of[r]] = recs[r][0]
        M0, M1, M2 = (max(x[i] for x in recs) for i in (1, 2, 3))
        deg = M0 if k == 0 else (M2 if M1 < 0 else M0)
        lvl = ordered
        while len(lvl) > 1:
            lvl = [hashlib.sha256(lvl[2 * i] + lvl[2 * i + 1]).digest() for i in range(len(lvl) // 2)]
        root = lvl[0]
        roots.append(root)
        ch.send(root.hex().encode())
        if deg < 1:
            final = 0 if deg == -1 else recs[0][4]               # poly_k[0] from rank 0's record
            ch.send(fo.fe_to_bytes(final))
            return {"roots": [r.hex() for r in roots], "betas": betas, "final_value": final,
                    "final_degree": deg, "state": ch.state}
        beta = ch.receive_random_field_element()
        betas.append(beta)
        m = 1 << Lk
        off_k = fo.fe_pow(offset, 1 << k, P)
        w_k = fo.fe_pow(5, (P - 1) // m, P)
        b = block_of[rank]
        isA = b < G // 2
        partner = block_of.index(b + G // 2) if isA else block_of.index(b - G // 2)
        if k < k_sw:
            mine = block[B // 2:] if isA else block[: B // 2]
            t_send = torch.from_numpy(mine.astype(np.int64).copy())
            t_recv = torch.empty_like(t_send)
            for req in dist.batch_isend_irecv([dist.P2POp(dist.isend, t_send, partner),
                                              dist.P2POp(dist.irecv, t_recv, partner)]):
                req.wait()
            half = t_recv.numpy().astype(np.uint64)
            bb = b if isA else b - G // 2
            first = block[: B // 2] if isA else half
            second = half if isA else block[B // 2:]
            base = bb * B + (0 if isA else B // 2)
            out = np.zeros(B // 2, dtype=np.uint64)
            for j in range(B // 2):
                x = fo.fe_mul(off_k, fo.fe_pow(w_k, base + j, P), P)
                a_, b_ = int(first[j]), int(second[j])
                v = (a_ + b_ + beta * ((a_ - b_) % P) * fo.fe_inverse(x, P)) % P
                out[j] = v * inv2 % P
            block = out
            block_of = [2 * br if br < G // 2 else 2 * (br - G // 2) + 1 for br in block_of]
            k += 1
            continue
        # switch to local: gather the full layer in block order and poly_k
        # (the chunks in rank order), then fold/commit locally
        parts = _allgather_u64(block, G)
        full = np.zeros(m, dtype=np.uint64)
        for r in range(G):
            full[block_of[r] * B:(block_of[r] + 1) * B] = parts[r]
        if k == 0:
            poly = list(coeffs[:deg + 1])
        else:
            mine = np.array([chunk.get(j, 0) for j in range(rank * Sk, (rank + 1) * Sk)], dtype=np.uint64)
            allc = np.concatenate(_allgather_u64(mine, G))
            poly = [int(x) for x in allc[:deg + 1]]
        poly, deg = fo.next_fri_polynomial(poly, deg, beta, P)
        cur = full
        while True:
            mm = cur.size
            h = mm // 2
            off_k = fo.fe_pow(offset, 1 << k, P)
            w_k = fo.fe_pow(5, (P - 1) // mm, P)
            nxt = np.zeros(h, dtype=np.uint64)
            for i in range(h):
                x = fo.fe_mul(off_k, fo.fe_pow(w_k, i, P), P)
                a_, b_ = int(cur[i]), int(cur[i + h])
                nxt[i] = (a_ + b_ + beta * ((a_ - b_) % P) * fo.fe_inverse(x, P)) % P * inv2 % P
            cur = nxt
            k += 1
            root = _tree_root(lib, cur)
            roots.append(root)
            ch.send(root.hex().encode())
            if deg < 1:
                final = 0 if deg == -1 else poly[0]
                ch.send(fo.fe_to_bytes(final))
                return {"roots": [r.hex() for r in roots], "betas": betas, "final_value": final,
                        "final_degree": deg, "state": ch.state}
            beta = ch.receive_random_field_element()
            betas.append(beta)
            poly, deg = fo.next_fri_polynomial(poly, deg, beta, P)
