"""Host check of the torch_rocm bf16 shortcut (fks_device.hip phx_z_bf16, DESIGN.md §6b'):
the kernel computes z' = RN_f32(sc * s') with the raw root s' (within 1 ulp of ocml's
correctly rounded s) and keeps bf16(z') unless z' lies within 4 f32 ulps of a bf16
rounding midpoint.  Here, for random (sc, s) and s' = s - 1 ulp, s, s + 1 ulp: whenever the
window test says "far", bf16(RN(sc * s')) == bf16(RN(sc * s)).  Products are exact in
float64 (24 x 24 bits), so the float32 cast is the correctly rounded product."""
import numpy as np

BF16_MASK = np.uint32(0xFFFF0000)


def rne_bf16(bits: np.ndarray) -> np.ndarray:
    """RNE to bf16 of float32 bit patterns (finite inputs), as v_cvt_pk_bf16_f32."""
    lsb = (bits >> np.uint32(16)) & np.uint32(1)
    return ((bits + np.uint32(0x7FFF) + lsb) & BF16_MASK).astype(np.uint32)


def near_mid(bits: np.ndarray) -> np.ndarray:
    """phx_near_bf16_mid: low 16 bits within [0x7FFC, 0x8004]."""
    return ((bits & np.uint32(0xFFFF)) - np.uint32(0x7FFC)) <= np.uint32(8)


def prod_f32(sc: np.ndarray, s: np.ndarray) -> np.ndarray:
    return (sc.astype(np.float64) * s.astype(np.float64)).astype(np.float32).view(np.uint32)


def ulp_step(s: np.ndarray, d: int) -> np.ndarray:
    return (s.view(np.uint32).astype(np.int64) + d).astype(np.uint32).view(np.float32)


def test_window_covers_every_one_ulp_radius_change():
    rng = np.random.default_rng(7)
    n = 1 << 21
    # radius over the torch_rocm domain: sqrt(-2 log u), u in [2^-32, 1]
    u = rng.random(n).astype(np.float64) * (1 - 2.0 ** -32) + 2.0 ** -32
    s = np.sqrt(-2.0 * np.log(u)).astype(np.float32)
    s = s[s > 0]
    sc = rng.uniform(-1.0, 1.0, s.size).astype(np.float32)  # sin / cos values
    sc[::97] = np.float32(1e-9)  # tiny angles' sines
    checked = 0
    for d in (-1, 1):
        z = prod_f32(sc, s)            # the exact-radius product
        zf = prod_f32(sc, ulp_step(s, d))  # the raw root one ulp off
        far = ~near_mid(zf)
        assert np.array_equal(rne_bf16(zf[far]), rne_bf16(z[far])), "a far product changed its bf16 rounding"
        checked += int(far.sum())
    assert checked > 0.99 * 2 * s.size  # the window takes about 9 / 65536 of the products


def test_products_next_to_a_midpoint_are_caught():
    # construct z' just around bf16 midpoints: the window must flag every one whose
    # neighbours within 3 ulps round differently
    rng = np.random.default_rng(8)
    hi = rng.integers(0x3000, 0x4100, 4096).astype(np.uint32) << np.uint32(16)
    for off in range(-8, 9):
        zf = hi | np.uint32(0x8000 + off)
        flips = np.zeros(zf.size, dtype=bool)
        for dz in range(-3, 4):
            flips |= rne_bf16((zf.astype(np.int64) + dz).astype(np.uint32)) != rne_bf16(zf)
        assert not np.any(flips & ~near_mid(zf)), f"offset {off}: a flip outside the window"
