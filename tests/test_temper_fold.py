"""The folded tempering index of the bf16 kernels (fks_device.hip temper_pair_u8x8,
FKS_TEMPER_FOLD): after the first two tempering steps of MT19937RNGEngine.h:141-145,
((y << 3) ^ (y >> 15) ^ (y & 0x788)) & 0x7F8 equals the full four-step tempering's low
byte times 8 -- checked here on random and structured words (host algebra, no GPU)."""
import numpy as np

U = np.uint32


def _temper_low8x8(y):
    y = y ^ (y >> U(11))
    y = y ^ ((y << U(7)) & U(0x9D2C5680))
    y = y ^ ((y << U(15)) & U(0xEFC60000))
    y = y ^ (y >> U(18))
    return (y & U(0xFF)) << U(3)


def _folded(y):
    y = y ^ (y >> U(11))
    y = y ^ ((y << U(7)) & U(0x9D2C5680))
    return (((y << U(3)) ^ (y >> U(15))) & U(0x7F8)) ^ (y & U(0x788))


def test_folded_index_equals_tempering():
    rng = np.random.default_rng(7)
    words = rng.integers(0, 2**32, size=1 << 22, dtype=np.uint64).astype(np.uint32)
    assert np.array_equal(_temper_low8x8(words), _folded(words))


def test_folded_index_on_single_bits():
    # linear over GF(2): agreeing on every basis vector and on 0 is agreeing everywhere
    basis = np.array([0] + [1 << i for i in range(32)], dtype=np.uint64).astype(np.uint32)
    assert np.array_equal(_temper_low8x8(basis), _folded(basis))
