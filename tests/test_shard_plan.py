"""CPU: the shard-sized commit plan (fri_commit.hip plan_layout, through the
host-only fri_debug_plan_layout; no GPU) against the protocol model.

Each rank of a G-way sharded commit allocates only its block of every sharded
layer and the x^-1 slice its fold reads.  Checked here for every rank:
  * the blocks held at each sharded layer follow the model's block
    permutation (tests/dist_model.py: the fold of blocks b and b + G/2 leaves
    2b and 2b + 1), and form a permutation of 0..G-1;
  * the x^-1 slices of all ranks' folds partition [0, n_k / 2) exactly;
  * slot sizes: blocks up to the switch layer, the full gathered layer at the
    switch when a local tail follows, full local layers after it;
  * per-rank bytes: ~168 n / G + the local tail at 2^28 over 8 ranks
    (the round-2 plan allocated the whole codeword's ~34 GB on every rank).
"""
import itertools

import pytest

import fri_amd

SHARD_MIN_LOG = 20


def model_blocks(G, n_layers):
    """block_of[r] per layer, as tests/dist_model.py evolves it."""
    block_of = list(range(G))
    out = []
    for _ in range(n_layers):
        out.append(list(block_of))
        block_of = [2 * b if b < G // 2 else 2 * (b - G // 2) + 1 for b in block_of]
    return out


def model_switch(log_n, logG, rmax):
    k = 0
    while k < rmax and (log_n - k - 1) >= SHARD_MIN_LOG and (log_n - k - 1 - logG) >= 10:
        k += 1
    return k


@pytest.mark.parametrize("G,log_n,blowup_log", list(itertools.product((2, 4, 8, 16), (20, 22, 25, 28), (3, 1, 0))))
def test_shard_plan_partitions(G, log_n, blowup_log):
    logG = G.bit_length() - 1
    d = (1 << log_n) >> blowup_log
    plans = [fri_amd.plan_layout(d, log_n, G, r) for r in range(G)]
    rmax = plans[0]["rmax"]
    k_sw = plans[0]["k_sw"]
    assert all(p["rmax"] == rmax and p["k_sw"] == k_sw for p in plans)
    assert k_sw == model_switch(log_n, logG, rmax)
    blocks = model_blocks(G, k_sw + 1)
    for k in range(k_sw + 1):
        L = log_n - k
        B = 1 << (L - logG)
        assert sorted(p["layers"][k]["block"] for p in plans) == list(range(G))
        for r, p in enumerate(plans):
            lay = p["layers"][k]
            assert lay["block"] == blocks[k][r]
            assert lay["tree_words"] == 8 * (2 * B - 1)            # block-local tree
            full = k == k_sw and k_sw < rmax                        # the gathered layer at the switch
            assert lay["layer_words"] == (1 << L if full else B)
        if k < k_sw:                                                # sharded fold: slices partition n_k / 2
            spans = sorted((p["layers"][k]["xinv_start"], p["layers"][k]["xinv_count"]) for p in plans)
            pos = 0
            for start, cnt in spans:
                assert start == pos and cnt == B // 2
                pos += cnt
            assert pos == (1 << L) // 2
    for p in plans:                                                 # local layers after the switch: full size
        for k in range(k_sw + 1, rmax + 1):
            L = log_n - k
            lay = p["layers"][k]
            assert lay["layer_words"] == 1 << L and lay["tree_words"] == 8 * ((2 << L) - 1)
        for k in range(k_sw, rmax):
            lay = p["layers"][k]
            assert lay["xinv_start"] == 0 and lay["xinv_count"] == (1 << (log_n - k)) // 2


def test_shard_plan_bytes_configs4():
    """BASELINE configs[4]: 2^28 over 8 ranks, ~5 GiB of plan per rank (plus
    the full coefficient vector and the context), against ~34 GB for the
    whole-codeword plan."""
    whole = fri_amd.plan_layout(1 << 25, 28)["bytes"]
    per_rank = [fri_amd.plan_layout(1 << 25, 28, 8, r)["bytes"] for r in range(8)]
    assert whole > 33 * 2**30
    assert max(per_rank) < whole / 8 + (256 << 20)
    assert len(set(per_rank)) == 1


def test_single_plan_layout():
    p = fri_amd.plan_layout(1 << 21, 24)
    assert p["rmax"] == 21 and p["k_sw"] == -1
    for k, lay in enumerate(p["layers"]):
        L = 24 - k
        assert lay["layer_words"] == 1 << L and lay["tree_words"] == 8 * ((2 << L) - 1)
        assert lay["xinv_count"] == ((1 << L) // 2 if k < 21 else 0)


@pytest.mark.parametrize("G,log_n", list(itertools.product((2, 4, 8, 16, 64), (20, 22, 25, 28, 30))))
@pytest.mark.parametrize("d_shape", ["n/8", "n", "odd", "tiny", "one", "zero"])
def test_coefficient_chunks_cover_every_round(G, log_n, d_shape):
    """The sharded coefficient fold (next_fri_polynomial, fri_commit.rs:32-50):
    rank r folds coefficients [r*S_k, (r+1)*S_k) of poly_k with S_k = S_0/2^k.
    The G chunks must cover every coefficient poly_k can have (ceil(d/2^k))
    in every sharded round, each chunk must hold at least one coefficient
    there (a pair c_2j, c_2j+1 of poly_{k-1} then never straddles two
    chunks), and S_0 is the smallest power of two that does both."""
    if log_n < (G.bit_length() - 1) + 12:
        pytest.skip("codeword too small for this world")
    n = 1 << log_n
    d = {"n/8": n >> 3, "n": n, "odd": (n >> 3) + 12345, "tiny": 5, "one": 1, "zero": 0}[d_shape]
    p = fri_amd.plan_layout(d, log_n, G, 0)
    S0, k_sw = 1 << p["coef_chunk_log2"], p["k_sw"]
    assert all(fri_amd.plan_layout(d, log_n, G, r)["coef_chunk_log2"] == p["coef_chunk_log2"] for r in (1, G - 1))
    for k in range(0, k_sw + 1):
        Sk = S0 >> k
        assert Sk >= 1 and Sk << k == S0
        assert G * Sk >= -(-d // (1 << k))            # every coefficient of poly_k has an owner
    minimal = S0 == 1 or (G * (S0 // 2) < d) or (S0 // 2 < (1 << k_sw))
    assert minimal, (S0, d, G, k_sw)
