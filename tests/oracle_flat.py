"""Test helper: a whole FRI transcript (commit + decommitment) from the C
oracle at sizes the Python twin cannot build trees for in seconds (2^20+).

orc_fri_commit_fast (oracle/fri_oracle.c, fri_commit.rs:72-122) writes every
layer and every tree level out; thin index views over those flat arrays are
handed to the Python twin's decommit_fri (fri_commit.rs:137-179), so the
decommitment messages come from the oracle's own code over the oracle's own
trees.  Test infrastructure only (like everything under oracle/)."""
import ctypes

import numpy as np

import fri_oracle as fo


class _Values:
    """Layer k's values as the twin indexes them (ints)."""

    def __init__(self, arr):
        self.a = arr

    def __len__(self):
        return int(self.a.size)

    def __getitem__(self, i):
        return int(self.a[i])


class _Level:
    """One tree level: digest j = 32 bytes at node offset + j."""

    def __init__(self, buf, off, cnt):
        self.buf, self.off, self.cnt = buf, off, cnt

    def __len__(self):
        return self.cnt

    def __getitem__(self, j):
        if not 0 <= j < self.cnt:
            raise IndexError(j)
        o = 32 * (self.off + j)
        return bytes(self.buf[o:o + 32])


def transcript(corc, coeffs, log_n, num_queries, max_index=None, offset=fo.GEN, state=""):
    """(proof messages, final channel state) of fri_commit followed by
    decommit_fri(num_queries, max_index) on the C oracle's layers and trees."""
    n = 1 << log_n
    c = np.ascontiguousarray(np.asarray(coeffs, dtype=np.uint64))
    sizes = []
    m = n
    while m >= 1:
        sizes.append(m)
        m >>= 1
    layers_out = np.zeros(sum(sizes), dtype=np.uint64)
    nodes = sum(corc.orc_merkle_nodes_count(s) for s in sizes)
    trees_out = ctypes.create_string_buffer(32 * nodes)
    och = fo.OrcChannel()
    corc.orc_channel_init(ctypes.byref(och))
    if state:
        och.state = state.encode()
        och.state_len = 64
    r = fo.OrcFriResult()
    rc = corc.orc_fri_commit_fast(c.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), c.size, log_n, offset, fo.GEN,
                                  fo.P, ctypes.byref(och), None, ctypes.byref(r),
                                  layers_out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), trees_out)
    assert rc == 0
    msgs = []
    for k in range(r.n_layers):
        msgs.append(bytes(r.roots[k]).hex().encode())
        if k < r.n_rounds:
            msgs.append(int(r.betas[k]).to_bytes(8, "big"))
    msgs.append(int(r.final_value).to_bytes(8, "big"))
    raw = memoryview(trees_out).cast("B")
    layers, trees = [], []
    lo, to = 0, 0
    for k in range(r.n_layers):
        m = n >> k
        layers.append(_Values(layers_out[lo:lo + m]))
        levels, off, cnt = [], to, m
        while True:
            levels.append(_Level(raw, off, cnt))
            if cnt == 1:
                break
            off += cnt
            cnt = (cnt + 1) // 2
        trees.append(levels)
        lo += m
        to += corc.orc_merkle_nodes_count(m)
    ch = fo.Channel(state=och.state.decode())
    ch.proof = list(msgs)
    fo.decommit_fri(num_queries, (n - 1) if max_index is None else max_index, layers, trees, ch)
    return ch.proof, ch.state
