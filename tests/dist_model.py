"""CPU model of the coset-sharded FRI commit (test infrastructure).

Mirrors run_commit_sharded (stark-prover_amd/csrc/fri_api.hip) step for step
with the same index math, using the C oracle for per-block work and
torch.distributed (gloo) for the exchanges:

  layer 0   rank r: P mod (x^M - s^M), s = offset*w_n^r, size-M LDE on s*<w_M>
            -> evals[r + G*m];  all-to-all of M/G chunks;  block[G*t + r] = recv[r][t]
  layer k   block-local Merkle tree; all-gather block roots; reorder by
            block_of; top log2(G) levels + channel (identical on every rank)
  fold      ranks holding blocks b and b + G/2 swap half-blocks; A keeps the
            first half of the outputs, B the second; block_of <- 2b / 2b'+1
  switch    below 2^shard_min_log: all-gather the layer, finish locally.
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
    poly = fo.poly_trim(coeffs)
    deg = len(poly) - 1
    roots, betas = [], []
    k = 0
    inv2 = fo.fe_inverse(2, P)
    while True:
        Lk = log_n - k
        B = 1 << (Lk - logG)
        rb = _tree_root(lib, block)
        got = _allgather_bytes(rb, G)
        ordered = [None] * G
        for r in range(G):
            ordered[block_of[r]] = got[r]
        lvl = ordered
        while len(lvl) > 1:
            lvl = [hashlib.sha256(lvl[2 * i] + lvl[2 * i + 1]).digest() for i in range(len(lvl) // 2)]
        root = lvl[0]
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
        m = 1 << Lk
        off_k = fo.fe_pow(offset, 1 << k, P)
        w_k = fo.fe_pow(5, (P - 1) // m, P)
        b = block_of[rank]
        isA = b < G // 2
        partner = block_of.index(b + G // 2) if isA else block_of.index(b - G // 2)
        if Lk - 1 >= shard_min_log and Lk - 1 - logG >= 1:
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
        # switch to local: gather the full layer in block order and fold/commit locally
        parts = _allgather_u64(block, G)
        full = np.zeros(m, dtype=np.uint64)
        for r in range(G):
            full[block_of[r] * B:(block_of[r] + 1) * B] = parts[r]
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
