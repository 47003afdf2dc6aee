"""Layout properties of the CQT kernels that no output test can see (they change speed, not
results), checked against a model of the hardware rules they were designed for:

* `xcd_remap` (nc_device.h) must be a permutation of the workgroup ids for every grid size,
  or workgroups would be skipped or run twice;
* the fragment reads of `cqt_mfma_kernel` (image pads `cm_pad`, or since round 5 the XOR
  swizzle `cm_phys` of hop-64 / hop-32 images, cqt.hip) and of
  `cqt_mfma_low_kernel` (image swizzle `c2_sw`, round 5) must be free of LDS bank conflicts under the
  `ds_read_b128` lane groups of MI355X_MICROARCH.md (LDS table): one LDS cycle per group.

The C++ rules are restated here; a change to either side has to change both."""
import pytest

# ds_read_b128: four groups of 16 lanes, bank of byte address a = (a / 4) mod 64
B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
               list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
               list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64))]


def b128_cycles(dword_addr):
    """LDS cycles of one wave-wide ds_read_b128 (4 when conflict free)."""
    total = 0
    for grp in B128_GROUPS:
        banks = {}
        for lane in grp:
            for d in range(4):
                a = dword_addr[lane] + d
                banks.setdefault(a % 64, set()).add(a)
        total += max(len(v) for v in banks.values())
    return total


def xcd_remap(l, n):  # nc_device.h
    q, r, x = n // 8, n % 8, l % 8
    return x * q + min(x, r) + l // 8


@pytest.mark.parametrize("n", [1, 7, 8, 9, 63, 64, 100, 768, 3136, 4705])
def test_xcd_remap_is_a_permutation(n):
    assert sorted(xcd_remap(l, n) for l in range(n)) == list(range(n))


def cm_hop(o):
    return 512 >> o


def cm_pad(o):  # cqt.hip, the padded layout of CH_SWZ_=0 builds (the default until round 5)
    return 16 if cm_hop(o) >= 32 else 0


@pytest.mark.parametrize("octave", [3, 4, 5, 6])
def test_octave_3_6_image_reads_conflict_free(octave):
    """A fragment: row 16 rt + (lane & 15) of the image, k offset 8 (lane >> 4) halves, rows
    hop + pad halves apart, a pad after every hop samples (cqt_mfma_kernel abase / kt)."""
    hop, pad = cm_hop(octave), cm_pad(octave)
    for rt in range(4):
        for ks in range(32):
            kt = 32 * ks + (32 * ks // hop) * pad
            halves = [(16 * rt + (l & 15)) * (hop + pad) + 8 * (l >> 4) + ((8 * (l >> 4)) // hop) * pad + kt
                      for l in range(64)]
            assert all(h % 8 == 0 for h in halves)  # 16-byte aligned pieces
            assert b128_cycles([h // 2 for h in halves]) == 4, (octave, rt, ks)


# cqt.hip cm_swz_k / cm_swz_m / cm_phys (the default since round 5): piece P of a hop-64 or hop-32
# image sits at P ^ h[(P >> 4) & m]; hop 16 and 8 are unpadded and unswizzled
CM_SWZ = {64: (0xC638, 3), 32: (0xF8, 1)}


def cm_phys(P, hop):
    if hop not in CM_SWZ:
        return P
    K, m = CM_SWZ[hop]
    return P ^ ((K >> (((P >> 4) & m) << 2)) & 15)


@pytest.mark.parametrize("frames", [32, 64])
@pytest.mark.parametrize("octave", [3, 4, 5, 6])
def test_octave_3_6_swizzled_image_reads_conflict_free(octave, frames):
    """Fragment of row tile rt at k-step ks: lane l reads piece (16 rt + (l & 15)) hop / 8 +
    l >> 4 + 4 ks through the swizzle (cqt_mfma_kernel abase / cm_phys)."""
    hop = cm_hop(octave)
    for rt in range(frames // 16):
        for ks in range(32):
            pieces = [cm_phys((16 * rt + (l & 15)) * hop // 8 + (l >> 4) + 4 * ks, hop) for l in range(64)]
            assert b128_cycles([4 * p for p in pieces]) == 4, (octave, rt, ks)


@pytest.mark.parametrize("frames", [32, 64])
@pytest.mark.parametrize("octave", [3, 4, 5, 6])
def test_octave_3_6_swizzle_is_a_permutation_inside_the_image(octave, frames):
    """Every piece of the span lands on a distinct piece of the image (cm_img: whole 256-byte
    blocks when swizzled), so no write overlaps another or leaves the octave's image."""
    hop = cm_hop(octave)
    span = (frames - 1) * hop + 1024
    img = (span + 127) & ~127 if hop in CM_SWZ else (span + 7) & ~7
    phys = [cm_phys(p, hop) for p in range(span // 8)]
    assert len(set(phys)) == len(phys) and max(phys) < img // 8


def test_octave_3_6_lds_fits_three_workgroups():
    """cqm_lds_bytes at 32 frames swizzled: ring (2 slots x 10 KB) + the four images (hi + lo)."""
    tot = 2 * 5 * 2 * 64 * 16
    for o in range(3, 7):
        hop = cm_hop(o)
        span = 31 * hop + 1024
        tot += 4 * ((span + 127) & ~127 if hop in CM_SWZ else (span + 7) & ~7)
    assert 3 * tot <= 160 * 1024, tot


SF_RS = 72  # spectral.hip spectral_frames_kernel: row stride (f64) of the frame-sum reduction


def test_spectral_frame_sum_reduction_conflict_free():
    """Writes red[v][lane] (ds_write_b64: 4 x 16 contiguous lanes, banks (a/4) mod 32) and reads
    red[lane >> 3][(lane & 7) + 8 i] (ds_read_b64: lanes 0-31 and 32-63, banks (a/4) mod 64)
    of spectral_frames_kernel each take one LDS cycle per lane group."""
    for v in range(8):
        for g in range(4):
            dw = [2 * (SF_RS * v + l) for l in range(16 * g, 16 * g + 16)]
            banks = [(d + k) % 32 for d in dw for k in range(2)]
            assert len(set(banks)) == 32, (v, g)
    for i in range(8):
        for half in range(2):
            dw = [2 * (SF_RS * (l >> 3) + (l & 7) + 8 * i) for l in range(32 * half, 32 * half + 32)]
            banks = [(d + k) % 64 for d in dw for k in range(2)]
            assert len(set(banks)) == 64, (i, half)
    # the eight rows fit the wave's FFT slot (LdsSize<1024> = 1056 float2)
    assert 8 * SF_RS * 8 <= 1056 * 8


# ---- cqt_mfma_low_kernel (round 5): per-wave f16 images, 64-byte rows of four 16-byte pieces
def c2_sw(R):  # cqt.hip
    return ((R >> 2) & 1) << 1


def c2_off(R, p):
    return R * 64 + 16 * (p ^ c2_sw(R))


@pytest.mark.parametrize("q", range(8))
@pytest.mark.parametrize("rt", range(4))
def test_low_octave_fragment_reads_conflict_free(q, rt):
    """A fragment of row tile rt at group position q: lane l reads row 16 rt + (l & 15) + q,
    piece l >> 4 (8 halves)."""
    addr = [c2_off(16 * rt + (lane & 15) + q, lane >> 4) // 4 for lane in range(64)]
    assert b128_cycles(addr) == 4


def b128_write_cycles(dword_addr):
    """ds_write_b128: eight groups of 8 consecutive lanes, bank (a / 4) mod 32."""
    total = 0
    for g in range(8):
        banks = {}
        for lane in range(8 * g, 8 * g + 8):
            for d in range(4):
                a = dword_addr[lane] + d
                banks.setdefault(a % 32, set()).add(a)
        total += max(len(v) for v in banks.values())
    return total


@pytest.mark.parametrize("k", range(5))
def test_low_octave_split_writes_conflict_free(k):
    """The split of staging round k: lane l writes unit u = 64 k + l (row u / 4, piece u % 4)."""
    addr = [c2_off((64 * k + lane) >> 2, (64 * k + lane) & 3) // 4 for lane in range(64)]
    assert b128_write_cycles(addr) == 8


def test_low_octave_images_hold_every_block_row():
    for o in range(3):
        H = 512 >> o
        M = 1024 // H
        assert 64 + M - 1 <= 72                          # C2_NRP
        assert 64 * ((72 * 4 + 63) // 64) >= 4 * (64 + M - 1)  # C2_NU staging rounds cover the rows
