"""Python face of the gfx950 health canary (``ops/canary.hip``).

``run(device)`` loads ``libamdgpu_canary.so`` with ctypes (no torch needed) and runs
the HBM pattern test, the MFMA exactness/throughput probe, the matrix-path check
(an LDS-staged MFMA GEMM on exact integer data with ABFT row/column checksums), the
fp8 / bf8 / fp4 MFMA exactness and rate checks and the LDS march (``datapath.hip``) on
one HIP device (= one compute partition).  ``run_isolated(device)`` does the same in a child process so the
long-lived plugin daemon never creates a HIP context on GPUs it hands to pods.

CLI: ``python -m k8s_gpu_device_plugin_amd.ops.canary --device 0 [--bytes N]`` prints
one JSON line.  Missing library => loud ``RuntimeError`` (never a silent pass).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libamdgpu_canary.so")


class CanaryResult(ctypes.Structure):
    _fields_ = [("ok", ctypes.c_int), ("device", ctypes.c_int), ("hbm_bytes", ctypes.c_ulonglong),
                ("hbm_errors", ctypes.c_ulonglong), ("mfma_errors", ctypes.c_ulonglong),
                ("write_gbps", ctypes.c_double), ("read_gbps", ctypes.c_double), ("mfma_tflops", ctypes.c_double),
                ("elapsed_ms", ctypes.c_double), ("num_cus", ctypes.c_int), ("arch", ctypes.c_char * 64),
                ("error", ctypes.c_char * 256), ("gemm_tflops", ctypes.c_double),
                ("gemm_errors", ctypes.c_ulonglong), ("fp8_tflops", ctypes.c_double),
                ("fp4_tflops", ctypes.c_double), ("lowp_errors", ctypes.c_ulonglong),
                ("lds_errors", ctypes.c_ulonglong), ("lds_bytes", ctypes.c_ulonglong)]


_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            from .. import _build
            _build.build_canary(verbose=False)
        lib = ctypes.CDLL(LIB_PATH)
        lib.amdgpu_canary_run.argtypes = [ctypes.c_int, ctypes.c_ulonglong, ctypes.c_int, ctypes.c_int,
                                          ctypes.POINTER(CanaryResult)]
        lib.amdgpu_canary_run.restype = ctypes.c_int
        lib.amdgpu_canary_device_count.restype = ctypes.c_int
        lib.amdgpu_canary_mfma_gemm.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                                                ctypes.c_int]
        lib.amdgpu_canary_mfma_gemm.restype = ctypes.c_int
        lib.amdgpu_canary_detects_corruption.argtypes = [ctypes.c_int, ctypes.c_ulonglong, ctypes.c_int]
        lib.amdgpu_canary_detects_corruption.restype = ctypes.c_longlong
        lib.amdgpu_canary_mfma_detects.argtypes = [ctypes.c_int, ctypes.c_int]
        lib.amdgpu_canary_mfma_detects.restype = ctypes.c_longlong
        lib.amdgpu_canary_hbm_sweep.argtypes = [ctypes.c_int, ctypes.c_ulonglong, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                                ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_ulonglong)]
        lib.amdgpu_canary_hbm_sweep.restype = ctypes.c_int
        lib.amdgpu_canary_gemm.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                                           ctypes.c_int]
        lib.amdgpu_canary_gemm.restype = ctypes.c_int
        lib.amdgpu_canary_gemm_rate.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                                ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_char_p, ctypes.c_int]
        lib.amdgpu_canary_gemm_rate.restype = ctypes.c_int
        lib.amdgpu_canary_lowp_check.argtypes = [ctypes.c_int] * 5
        lib.amdgpu_canary_lowp_check.restype = ctypes.c_longlong
        lib.amdgpu_canary_lowp_rate.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                ctypes.POINTER(ctypes.c_double)]
        lib.amdgpu_canary_lowp_rate.restype = ctypes.c_int
        lib.amdgpu_canary_lds_check.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_ulonglong)]
        lib.amdgpu_canary_lds_check.restype = ctypes.c_longlong
        lib.amdgpu_canary_lowp_gemm.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 5 + \
            [ctypes.c_int] * 3 + [ctypes.c_char_p, ctypes.c_int]
        lib.amdgpu_canary_lowp_gemm.restype = ctypes.c_int
        _lib = lib
    return _lib


def device_count() -> int:
    return load().amdgpu_canary_device_count()


def run(device: int = 0, hbm_bytes: int = 1 << 30, passes: int = 3, mfma_iters: int = 8192) -> dict:
    r = CanaryResult()
    rc = load().amdgpu_canary_run(int(device), int(hbm_bytes), int(passes), int(mfma_iters), ctypes.byref(r))
    out = {f[0]: getattr(r, f[0]) for f in CanaryResult._fields_}
    out["arch"] = r.arch.decode(errors="replace")
    out["error"] = r.error.decode(errors="replace")
    out["ok"] = bool(r.ok) and rc == 0
    return out


def detects_corruption(device: int = 0, hbm_bytes: int = 64 << 20, flips: int = 5) -> int:
    """Fault-injection check of the HBM verifier; returns the mismatches it found."""
    return int(load().amdgpu_canary_detects_corruption(int(device), int(hbm_bytes), int(flips)))


def mfma_detects_corruption(device: int = 0, inject_blocks: int = 3) -> int:
    """Fault-injection check of the MFMA exactness verifier; returns the wrong
    accumulator registers it found (0 expected with inject_blocks=0)."""
    return int(load().amdgpu_canary_mfma_detects(int(device), int(inject_blocks)))


# cbsz/blgp format codes of v_mfma_scale_f32_32x32x64_f8f6f4 (OCP formats); "fp8_unscaled" is
# v_mfma_f32_32x32x16_fp8_fp8
LOWP_FORMATS = {"fp8": 0, "bf8": 1, "fp4": 4, "fp8_unscaled": 8}


def lowp_check(device: int = 0, fmt: str = "fp8", ksteps: int = 4, vary_scale: bool = True,
               inject_blocks: int = 0) -> int:
    """Exactness of one low-precision MFMA form on small-integer operands with power-of-two
    block scales (2 single-wave blocks per CU, K = 64 * ksteps); returns the wrong
    accumulator registers (0 expected unless ``inject_blocks`` perturb an operand)."""
    rc = load().amdgpu_canary_lowp_check(int(device), LOWP_FORMATS[fmt], int(ksteps), int(bool(vary_scale)),
                                         int(inject_blocks))
    if rc < 0:
        raise RuntimeError("lowp_check(%s) failed on device %d" % (fmt, device))
    return int(rc)


def lowp_rate(device: int = 0, fmt: str = "fp8", iters: int = 2048) -> float:
    """Dense TFLOP/s of the block-scaled MFMA on ``fmt`` (fp8, bf8 or fp4)."""
    t = ctypes.c_double()
    if load().amdgpu_canary_lowp_rate(int(device), LOWP_FORMATS[fmt], int(iters), ctypes.byref(t)) != 0:
        raise RuntimeError("lowp_rate(%s) failed on device %d" % (fmt, device))
    return t.value


def lds_check(device: int = 0, inject_blocks: int = 0) -> tuple:
    """LDS march over every CU's whole LDS; returns (mismatches, bytes per workgroup)."""
    nbytes = ctypes.c_ulonglong()
    rc = load().amdgpu_canary_lds_check(int(device), int(inject_blocks), ctypes.byref(nbytes))
    if rc < 0:
        raise RuntimeError("lds_check failed on device %d" % device)
    return int(rc), int(nbytes.value)


def lowp_gemm(a_codes, bt_codes, a_scales, b_scales, fmt: str = "fp8", device: int = 0):
    """C = dequant(A) @ dequant(Bt).T through the block-scaled MFMA.  ``a_codes`` uint8 [M, K]
    and ``bt_codes`` uint8 [N, K] hold one OCP code per element (fp4 in the low nibble);
    ``a_scales`` [M, K/32], ``b_scales`` [N, K/32] are E8M0 exponents (127 = 1.0).
    M, N % 32 == 0, K % 64 == 0.  Returns float32 [M, N]."""
    import numpy as np

    a = np.ascontiguousarray(a_codes, dtype=np.uint8)
    bt = np.ascontiguousarray(bt_codes, dtype=np.uint8)
    sa = np.ascontiguousarray(a_scales, dtype=np.uint8)
    sb = np.ascontiguousarray(b_scales, dtype=np.uint8)
    (m, k), (nn, k2) = a.shape, bt.shape
    if k != k2 or sa.shape != (m, k // 32) or sb.shape != (nn, k // 32):
        raise ValueError("shapes do not match: A %s, Bt %s, scales %s / %s" % (a.shape, bt.shape, sa.shape, sb.shape))
    c = np.empty((m, nn), dtype=np.float32)
    err = ctypes.create_string_buffer(256)
    rc = load().amdgpu_canary_lowp_gemm(int(device), LOWP_FORMATS[fmt], a.ctypes.data, bt.ctypes.data,
                                        sa.ctypes.data, sb.ctypes.data, c.ctypes.data, m, nn, k, err, 256)
    if rc != 0:
        raise RuntimeError("lowp_gemm failed: " + err.value.decode(errors="replace"))
    return c


SWEEP_VARIANTS = {0: "u4 grid-stride", 1: "u8 grid-stride", 2: "u4 nontemporal", 3: "u8 nontemporal",
                  4: "u4 chunked", 5: "u8 chunked", 6: "u4 nt chunked", 7: "u16 grid-stride",
                  8: "u8 nt chunked", 9: "u2 nt chunked", 10: "u4 tile-stride (nt verify)",
                  11: "u8 tile-stride (nt verify)", 12: "u8 tile-stride"}


def hbm_sweep(device: int = 0, nbytes: int = 4 << 30, variants=tuple(SWEEP_VARIANTS), blocks_per_cu=(4, 8, 16),
              reps: int = 5) -> list:
    """Times write+verify for each access shape; returns rows of GB/s (HBM-resident buffer)."""
    rows = []
    for v in variants:
        for b in blocks_per_cu:
            w, r, e = ctypes.c_double(), ctypes.c_double(), ctypes.c_ulonglong()
            rc = load().amdgpu_canary_hbm_sweep(device, nbytes, v, b, reps, ctypes.byref(w), ctypes.byref(r),
                                                ctypes.byref(e))
            rows.append({"variant": SWEEP_VARIANTS[v], "blocks_per_cu": b, "write_gbps": round(w.value, 1),
                         "read_verify_gbps": round(r.value, 1), "errors": e.value, "rc": rc})
    return rows


def mfma_gemm(a_bf16_bits, b_bf16_bits, device: int = 0):
    """C = A @ B through the canary's MFMA kernel.  ``a``/``b``: uint16 numpy arrays of
    bf16 bit patterns (row-major, M,N % 32 == 0, K % 16 == 0); returns float32 [M, N]."""
    import numpy as np

    a = np.ascontiguousarray(a_bf16_bits, dtype=np.uint16)
    b = np.ascontiguousarray(b_bf16_bits, dtype=np.uint16)
    (m, k), (k2, nn) = a.shape, b.shape
    if k != k2:
        raise ValueError("inner dimensions differ: %d vs %d" % (k, k2))
    c = np.empty((m, nn), dtype=np.float32)
    err = ctypes.create_string_buffer(256)
    rc = load().amdgpu_canary_mfma_gemm(int(device), a.ctypes.data, b.ctypes.data, c.ctypes.data, m, nn, k, err, 256)
    if rc != 0:
        raise RuntimeError("mfma_gemm failed: " + err.value.decode(errors="replace"))
    return c


# kernel ids of amdgpu_canary_gemm*: "auto" picks pingpong256s for >= 256 tiles of 256x256, else lds128; the
# pingpong256s_* entries are the ablations in profiles/gemm_r1/SUMMARY.md
GEMM_KERNELS = {"auto": 0, "lds128": 1, "pingpong256": 2, "pingpong256s": 3, "pingpong256s_b2": 4,
                "pingpong256s_b0": 5, "pingpong256s_b3": 6, "pingpong256s_g1early": 7, "pingpong256s_vwave": 8,
                "pingpong256s_group2": 9, "pingpong256s_group8": 10, "pingpong256s_noprio": 11}


def gemm(a_bf16_bits, bt_bf16_bits, device: int = 0, kernel: str = "auto"):
    """C = A @ Bt.T through the LDS-staged MFMA GEMM (the canary's matrix path).
    ``a``: uint16 [M, K] bf16 bit patterns, ``bt``: uint16 [N, K] (B transposed, K
    contiguous); K % 64 == 0 and M, N % 128 == 0 (``lds128``) or % 256 == 0
    (``pingpong256``; ``auto`` takes it when that gives >= 256 tiles).  Returns float32
    [M, N]."""
    import numpy as np

    a = np.ascontiguousarray(a_bf16_bits, dtype=np.uint16)
    bt = np.ascontiguousarray(bt_bf16_bits, dtype=np.uint16)
    (m, k), (nn, k2) = a.shape, bt.shape
    if k != k2:
        raise ValueError("inner dimensions differ: %d vs %d" % (k, k2))
    c = np.empty((m, nn), dtype=np.float32)
    err = ctypes.create_string_buffer(256)
    rc = load().amdgpu_canary_gemm(int(device), a.ctypes.data, bt.ctypes.data, c.ctypes.data, m, nn, k,
                                   GEMM_KERNELS[kernel], err, 256)
    if rc != 0:
        raise RuntimeError("gemm failed: " + err.value.decode(errors="replace"))
    return c


def gemm_rate(device: int = 0, m: int = 4096, n: int = 4096, k: int = 4096, iters: int = 10,
              inject: bool = False, kernel: str = "auto", random_data: bool = False) -> dict:
    """Matrix-path canary: timed LDS-staged MFMA GEMMs on exact integer data, then ABFT
    row/column checksums.  ``errors`` counts rows + columns whose checksum is off.
    ``random_data``: uniform bf16 operands in [-1, 1) instead (the rate a BLAS benchmark
    quotes; no checksum, ``errors`` is None)."""
    t, e = ctypes.c_double(), ctypes.c_ulonglong()
    err = ctypes.create_string_buffer(256)
    rc = load().amdgpu_canary_gemm_rate(int(device), m, n, k, iters, int(bool(inject)) | (2 if random_data else 0),
                                        GEMM_KERNELS[kernel],
                                        ctypes.byref(t),
                                        ctypes.byref(e), err, 256)
    if rc != 0:
        raise RuntimeError("gemm_rate failed: " + err.value.decode(errors="replace"))
    return {"tflops": t.value, "errors": None if random_data else e.value, "shape": (m, n, k), "iters": iters,
            "kernel": kernel, "data": "random" if random_data else "integer"}


def run_isolated(device: int, hbm_bytes: int = 256 << 20, timeout: float = 120.0, passes: int = 1) -> dict:
    """``run`` in a child process (its own HIP runtime, gone when it exits)."""
    cmd = [sys.executable, "-m", "k8s_gpu_device_plugin_amd.ops.canary", "--device", str(device),
           "--bytes", str(hbm_bytes), "--passes", str(passes)]
    env = dict(os.environ)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
    try:
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout, env=env)
    except subprocess.TimeoutExpired:
        return {"ok": False, "device": device, "error": "canary timed out after %.0fs" % timeout}
    for line in reversed(p.stdout.strip().splitlines()):
        try:
            res = json.loads(line)
        except ValueError:
            continue
        if isinstance(res, dict):  # the result line, not stray output that happens to parse
            if p.returncode != 0 and res.get("ok"):
                res = dict(res, ok=False, error="canary reported ok but exited %d: %s"
                           % (p.returncode, p.stderr[-300:]))
            return res
    return {"ok": False, "device": device, "error": "canary exited %d: %s" % (p.returncode, p.stderr[-500:])}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="MI355X partition health canary")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--mfma-iters", type=int, default=8192)
    ap.add_argument("--gemm", type=int, default=0, help="only the matrix-path GEMM, at this M=N=K")
    ap.add_argument("--gemm-iters", type=int, default=20)
    ap.add_argument("--gemm-kernel", choices=sorted(GEMM_KERNELS), default="auto")
    ap.add_argument("--gemm-random", action="store_true", help="random bf16 operands (rate only, no checksum)")
    a = ap.parse_args(argv)
    if a.gemm:
        res = gemm_rate(a.device, a.gemm, a.gemm, a.gemm, a.gemm_iters, kernel=a.gemm_kernel,
                        random_data=a.gemm_random)
        print(json.dumps(res))
        return 0 if not res["errors"] else 1
    res = run(a.device, a.bytes, a.passes, a.mfma_iters)
    print(json.dumps(res))
    return 0 if res["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
