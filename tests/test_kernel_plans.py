"""Host-side launch plans of the round-4 kernels (CPU: the library's planning functions run
without a GPU).  The GPU numerics of the same paths are in test_hip_step.py /
test_deterministic.py (@gpu)."""
import pytest

from cloud_server_amd.ops import fused as K


@pytest.fixture(scope="module")
def lib():
    lib = K.load(required=False)
    if lib is None:
        pytest.skip("kernel library not built")
    lib.csa_set_deterministic(0)
    lib.csa_set_packed(0)
    yield lib
    lib.csa_set_deterministic(0)
    lib.csa_set_packed(0)


# the sample pair: conv 2x2x10 -> conv 2x2x20 -> 2x2 pool on 28x28x1 (TF SAME), B = 50
SAMPLE_PAIR = [50, 28, 28, 1, 2, 2, 0, 0, 10, 28, 28, 2, 2, 0, 0, 20, 28, 28, 1, 14, 14]


def test_pair_backward_tables_fit_the_prologue(lib):
    """One table region per band, each within the prologue's register batch (4 ints per
    thread of 256), in both launch profiles."""
    for packed in (0, 1):
        lib.csa_set_packed(packed)
        assert lib.csa_conv_pair_ok(K.ints(SAMPLE_PAIR))
        n = lib.csa_conv_pair_bwd_tables_size(K.ints(SAMPLE_PAIR))
        assert 0 < n <= 4 * 256 * 14, n
        assert n % 4 == 0
    lib.csa_set_packed(0)


def test_deterministic_rows_are_one_per_workgroup(lib):
    """Deterministic mode gives every statistic-producing workgroup its own slab row."""
    geom = [50, 14, 14, 20, 3, 3, 1, 1, 1, 1, 14, 14, 8]     # conv 3x3 20 -> 8, SAME, stride 1
    pool = [0, 1, 1, 1, 1, 0, 0, 14, 14]
    lib.csa_set_deterministic(0)
    assert lib.csa_conv_fwd_nslab(K.ints(geom), K.ints(pool)) == 32
    assert lib.csa_conv_dgrad_nslab(K.ints(geom)) == 32
    assert lib.csa_bn_stat_rows(50 * 14 * 14) == 16
    lib.csa_set_deterministic(1)
    try:
        fwd = lib.csa_conv_fwd_nslab(K.ints(geom), K.ints(pool))
        dgr = lib.csa_conv_dgrad_nslab(K.ints(geom))
        assert fwd >= 50 and fwd % 50 == 0        # one row per (image, band) workgroup
        assert dgr >= 50 and dgr % 50 == 0
        assert lib.csa_bn_stat_rows(50 * 14 * 14) == -(-50 * 14 * 14 // 64)
        wg = lib.csa_conv_wgrad_blocks(K.ints(geom), 1)
        assert wg >= 50 and wg % 50 == 0
    finally:
        lib.csa_set_deterministic(0)
