"""Pin the oracle: known-answer tests from the reference tree and from the
published test suites of its un-vendored RS dependency (reed-solomon-erasure 6.0.0,
which restates Backblaze JavaReedSolomon's tests).  CPU only."""
import numpy as np
import pytest


# ---- reed-solomon-erasure 6.0.0 galois_8 / ReedSolomon KATs (upstream test suite) ----
def test_galois8_mul_kats(oracle_mod):
    O = oracle_mod
    assert O.gf_mul(3, 4) == 12
    assert O.gf_mul(7, 7) == 21
    assert O.gf_mul(23, 45) == 41


def test_galois8_exp_kats(oracle_mod):
    O = oracle_mod
    assert O.gf_exp(2, 2) == 4
    assert O.gf_exp(5, 20) == 235
    assert O.gf_exp(13, 7) == 43


def test_galois8_field_axioms(oracle_mod):
    O = oracle_mod
    for a in range(1, 256):
        assert O.gf_mul(a, O.gf_inv(a)) == 1
        assert O.gf_div(O.gf_mul(a, 77), 77) == a
    assert O.gf_mul(0, 9) == 0 and O.gf_div(0, 9) == 0


def test_rs_5_5_one_encode_kat(oracle_mod):
    """reed-solomon-erasure test_one_encode / JavaReedSolomon testOneEncode."""
    shards = [[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]] + [[0, 0]] * 5
    out = oracle_mod.rs_encode(5, 5, shards)
    assert out[5:] == [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]]


def test_rs_systematic_and_mds(oracle_mod):
    rng = np.random.default_rng(0)
    for data, parity in [(4, 2), (9, 3), (12, 4), (10, 3)]:
        g = oracle_mod.rs_matrix(data, parity)
        assert np.array_equal(g[:data], np.eye(data, dtype=np.uint8))
        # any `data` rows invertible (MDS): reconstruct random erasure patterns
        shards = [list(rng.integers(0, 256, 8)) for _ in range(data)] + [[0] * 8] * parity
        enc = oracle_mod.rs_encode(data, parity, shards)
        assert enc[:data] == [list(map(int, s)) for s in shards[:data]]


def test_rs_generator_rows_of_clay_configs(oracle_mod):
    """Parity rows used by the BASELINE configs."""
    assert oracle_mod.rs_matrix(4, 2)[4:].tolist() == [[27, 28, 18, 20], [28, 27, 20, 18]]
    assert oracle_mod.rs_matrix(9, 3)[9:].tolist() == [
        [158, 158, 137, 137, 247, 247, 225, 225, 1],
        [160, 183, 160, 183, 33, 55, 33, 55, 1],
        [41, 62, 62, 41, 192, 214, 214, 192, 1]]
    assert oracle_mod.rs_matrix(12, 4)[12:].tolist() == [
        [175, 180, 150, 140, 245, 232, 196, 216, 27, 28, 18, 20],
        [180, 175, 140, 150, 232, 245, 216, 196, 28, 27, 20, 18],
        [150, 140, 175, 180, 196, 216, 245, 232, 18, 20, 27, 28],
        [140, 150, 180, 175, 216, 196, 232, 245, 20, 18, 28, 27]]


# ---- reference in-tree KATs ----
def test_transforms_kats(oracle_mod):
    """transforms.rs:163-225."""
    O = oracle_mod
    assert O.gf_mul(2, 2) != 1 and 2 != 0                      # test_gamma_properties
    assert O.gf_add(5, 3) == 6 and O.gf_mul(2, 3) == 6         # test_gf_arithmetic
    assert O.gf_mul(O.gf_inv(2), 2) == 1
    c, cs = [0x12, 0x34, 0x56, 0x78], [0xAB, 0xCD, 0xEF, 0x01]
    u, us = O.prt(c, cs)                                       # test_prt_pft_roundtrip
    assert O.pft(u, us) == (c, cs)
    assert O.gf_inv(1 ^ O.gf_mul(2, 2)) == 0xA7 and O.gf_inv(2) == 0x8E


def test_partial_transform_roundtrips(oracle_mod):
    """transforms.rs:192-213: the partial transforms agree with the full PRT / PFT."""
    O = oracle_mod
    c, cs = [0x12, 0x34, 0x56, 0x78], [0xAB, 0xCD, 0xEF, 0x01]
    u, us = O.prt(c, cs)                      # full PRT: (C, C*) -> (U, U*)
    assert O.c_from_u_and_cstar(u, cs) == c   # given U and C*, recover C
    assert O.u_from_c_and_ustar(c, us) == u   # given C and U*, recover U
    assert O.pft(u, us) == (c, cs)            # and the PFT round trip


def test_plane_vector_kats(oracle_mod):
    """coords.rs:42-61."""
    pv = oracle_mod.plane_vector
    assert pv(0, 2, 2) == [0, 0] and pv(1, 2, 2) == [0, 1]
    assert pv(2, 2, 2) == [1, 0] and pv(3, 2, 2) == [1, 1]
    assert pv(5, 2, 3) == [1, 2]


def test_max_iscore_kats(oracle_mod):
    """decode.rs:627-651."""
    c = oracle_mod.OracleClay(4, 2, 5)
    assert c.max_iscore([]) == 0
    assert c.max_iscore([0]) == 1
    assert c.max_iscore([0, 1]) == 1
    assert c.max_iscore([0, 2]) == 2
    assert c.max_iscore([0, 2, 4]) == 3  # one erasure in each of the t=3 y-sections


def test_companion_layer_range(oracle_mod):
    """decode.rs:596-616."""
    c = oracle_mod.OracleClay(4, 2, 5)
    for z in range(c.sub_chunk_no):
        zv = oracle_mod.plane_vector(z, c.t, c.q)
        for y in range(c.t):
            for x in range(c.q):
                assert c.companion_layer(z, x, y, zv[y]) < c.sub_chunk_no


def test_checked_pow(oracle_mod):
    """lib.rs:575-581."""
    assert oracle_mod.checked_pow(2, 63) is not None
    assert oracle_mod.checked_pow(2, 64) is None
    assert oracle_mod.checked_pow(10, 20) is None


@pytest.mark.parametrize("k,m,d,q,t,alpha,beta", [(4, 2, 5, 2, 3, 8, 4), (10, 4, 13, 4, 4, 256, 64),
                                                   (9, 3, 11, 3, 4, 81, 27)])
def test_parameters(oracle_mod, k, m, d, q, t, alpha, beta):
    """lib.rs:321-335, tests/integration.rs:13-19."""
    c = oracle_mod.OracleClay(k, m, d)
    assert (c.q, c.t, c.sub_chunk_no, c.beta) == (q, t, alpha, beta)


def test_repair_subchunk_counts(oracle_mod):
    """repair.rs:441-461."""
    c = oracle_mod.OracleClay(4, 2, 5)
    for lost in range(c.n):
        assert len(c.repair_subchunk_indices(lost if lost < c.k else lost + c.nu)) == c.beta
