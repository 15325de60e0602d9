"""Low-precision MFMA datapaths and LDS of the gfx950 canary (``ops/datapath.hip``), on a
real MI355X: exactness of the block-scaled fp8 / bf8 / fp4 and the unscaled fp8 MFMA, a
numerics check of the block-scaled GEMM against a PyTorch fp32 reference, the verifiers'
fault injection, the LDS march and the per-format MFMA rates."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FP4_VALUES = np.array([0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0], dtype=np.float32)


def _decode(codes, fmt):
    """OCP code -> float32 (no NaN/Inf codes are generated)."""
    import torch

    if fmt == "fp4":
        mag = FP4_VALUES[codes & 7]
        return torch.from_numpy(np.where(codes & 8, -mag, mag).astype(np.float32))
    dt = torch.float8_e4m3fn if fmt == "fp8" else torch.float8_e5m2
    return torch.from_numpy(np.ascontiguousarray(codes, dtype=np.uint8)).view(dt).float()


def _random_codes(rng, shape, fmt):
    if fmt == "fp4":
        return rng.integers(0, 16, size=shape, dtype=np.uint8)
    c = rng.integers(0, 256, size=shape, dtype=np.uint8)
    if fmt == "fp8":  # e4m3fn: S.1111.111 is NaN
        bad = (c & 0x7F) == 0x7F
    else:  # e5m2: exponent 11111 is Inf/NaN
        bad = (c & 0x7C) == 0x7C
    return np.where(bad, c & 0x83, c).astype(np.uint8)


@pytest.mark.parametrize("fmt", ["fp8", "bf8", "fp4", "fp8_unscaled"])
def test_lowp_mfma_exact_with_unit_scales(fmt):
    from k8s_gpu_device_plugin_amd.ops import canary
    assert canary.lowp_check(0, fmt, ksteps=4, vary_scale=False) == 0


@pytest.mark.parametrize("fmt", ["fp8", "bf8", "fp4"])
def test_lowp_mfma_exact_with_block_scales(fmt):
    """Per-lane E8M0 scales of 2^0 / 2^1 on A and B: lane (r, h)'s scale covers k-block h
    of row r, which for fp8/bf8 is spread over both lane halves (datapath.hip layout note,
    profiles/r2/lowp_layout_probe.json)."""
    from k8s_gpu_device_plugin_amd.ops import canary
    assert canary.lowp_check(0, fmt, ksteps=4, vary_scale=True) == 0


@pytest.mark.parametrize("fmt", ["fp8", "bf8", "fp4", "fp8_unscaled"])
def test_lowp_verifier_catches_injected_fault(fmt):
    from k8s_gpu_device_plugin_amd.ops import canary
    assert canary.lowp_check(0, fmt, ksteps=2, vary_scale=fmt != "fp8_unscaled", inject_blocks=3) > 0


@pytest.mark.parametrize("fmt", ["fp8", "bf8", "fp4"])
@pytest.mark.parametrize("shape", [(32, 32, 64), (64, 96, 256), (128, 64, 512)])
def test_lowp_gemm_matches_torch_fp32(fmt, shape):
    """Random codes over each format's whole finite range and random block scales against
    the fp32 GEMM of the dequantised operands.  fp4 products are small and the MFMA result
    matches to summation-order rounding.  The 8-bit forms do not compute an exact dot
    product: measured on MI355X, the result deviates by up to ~2^-11.4 of the largest
    product, unbiased, <= 1.8e-4 of sum|a*b| (fits neither fixed-point alignment nor a
    rounding adder tree of 10-16 bits; data in profiles/r2/lowp_numerics.md), so they get
    1e-3.  A wrong operand or scale layout is off by O(1)."""
    import torch

    from k8s_gpu_device_plugin_amd.ops import canary
    m, nn, k = shape
    rng = np.random.default_rng(m * 1000 + nn * 10 + k + len(fmt))
    a = _random_codes(rng, (m, k), fmt)
    bt = _random_codes(rng, (nn, k), fmt)
    sa = rng.integers(124, 131, size=(m, k // 32), dtype=np.uint8)
    sb = rng.integers(124, 131, size=(nn, k // 32), dtype=np.uint8)
    c = canary.lowp_gemm(a, bt, sa, sb, fmt=fmt, device=0)
    af = _decode(a, fmt) * torch.from_numpy(np.exp2(sa.astype(np.float32) - 127)).repeat_interleave(32, dim=1)
    bf = _decode(bt, fmt) * torch.from_numpy(np.exp2(sb.astype(np.float32) - 127)).repeat_interleave(32, dim=1)
    ref = (af @ bf.T).numpy()
    scale = (af.abs() @ bf.abs().T).numpy()
    err = np.abs(c - ref) / np.maximum(scale, 1e-30)
    assert err.max() < (1e-5 if fmt == "fp4" else 1e-3), (err.max(), np.unravel_index(err.argmax(), err.shape))


def test_lds_march_and_its_fault_injection():
    from k8s_gpu_device_plugin_amd.ops import canary
    bad, nbytes = canary.lds_check(0, 0)
    print("LDS march: %d bytes per workgroup, %d mismatches" % (nbytes, bad))
    assert bad == 0
    assert nbytes >= 64 * 1024
    bad, _ = canary.lds_check(0, 5)
    assert bad == 5  # one flipped bit in each of 5 workgroups


def test_lowp_mfma_rates():
    """Block-scaled fp8 runs at 2x and fp4 at 4x the bf16 MFMA rate per clock
    (MI355X_MICROARCH.md, matrix cores); the clock under MFMA load is below the boost
    clock, so the bounds are loose."""
    from k8s_gpu_device_plugin_amd.ops import canary
    bf16 = canary.run(0, hbm_bytes=64 << 20, passes=1, mfma_iters=8192)["mfma_tflops"]
    fp8 = canary.lowp_rate(0, "fp8", 2048)
    bf8 = canary.lowp_rate(0, "bf8", 2048)
    fp4 = canary.lowp_rate(0, "fp4", 4096)
    print("dense MFMA TFLOP/s: bf16 %.0f, fp8 %.0f, bf8 %.0f, fp4 %.0f" % (bf16, fp8, bf8, fp4))
    assert fp8 > 1.4 * bf16 and bf8 > 1.4 * bf16
    assert fp4 > 1.4 * fp8


def test_canary_run_covers_datapaths():
    from k8s_gpu_device_plugin_amd.ops import canary
    r = canary.run(0, hbm_bytes=256 << 20, passes=1, mfma_iters=4096)
    print("canary", {k: r[k] for k in ("fp8_tflops", "fp4_tflops", "lowp_errors", "lds_errors", "lds_bytes")})
    assert r["ok"], r
    assert r["lowp_errors"] == 0 and r["lds_errors"] == 0 and r["lds_bytes"] >= 64 * 1024
    assert r["fp8_tflops"] > 0 and r["fp4_tflops"] > 0
