"""Probes the operand / scale layout of v_mfma_scale_f32_32x32x64_f8f6f4 on the GPU with
raw fragments (``amdgpu_canary_lowp_raw``): which (lane, element) slots of A pair with
which of B, and which slots each lane's E8M0 scale multiplies.  Prints a JSON summary."""
import ctypes
import json
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from k8s_gpu_device_plugin_amd.ops import canary  # noqa: E402

ONE = {"fp8": 0x38, "bf8": 0x3C, "fp4": 0x2}
FMT = {"fp8": 0, "bf8": 1, "fp4": 4}


def raw(fmt, a, b, sa, sb):
    lib = canary.load()
    lib.amdgpu_canary_lowp_raw.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 5
    c = np.zeros((32, 32), dtype=np.float32)
    a, b = np.ascontiguousarray(a, np.uint8), np.ascontiguousarray(b, np.uint8)
    sa, sb = np.ascontiguousarray(sa, np.uint8), np.ascontiguousarray(sb, np.uint8)
    rc = lib.amdgpu_canary_lowp_raw(0, FMT[fmt], a.ctypes.data, b.ctypes.data, sa.ctypes.data, sb.ctypes.data,
                                    c.ctypes.data)
    assert rc == 0
    return c


def main():
    out = {}
    for fmt in ("fp8", "fp4"):
        one = ONE[fmt]
        res = {}
        # 1. slot pairing: A row r has a single 1 at slot (h, j); B column c has a single 1 at
        #    slot (h', j').  C[r][c] = 1 iff the hardware pairs them.
        pair_ok = True
        for (h, j) in [(0, 0), (0, 5), (0, 17), (1, 3), (1, 31)]:
            a = np.zeros((64, 32), np.uint8)
            b = np.zeros((64, 32), np.uint8)
            a[h * 32 + 0, j] = one          # row 0, slot (h, j)
            b[h * 32 + 7, j] = one          # column 7, same slot
            c = raw(fmt, a, b, np.full(64, 127), np.full(64, 127))
            pair_ok &= c[0, 7] == 1.0 and c.sum() == 1.0
        res["same_slot_pairs"] = bool(pair_ok)
        # 2. scale coverage: A = all ones, B column c has a 1 only at slot (hb, c)
        #    (c < 32); doubling lane L's A scale shows in C[row][c] for the slots it covers.
        cover = {}
        for lane in (0, 5, 32, 37):
            covered = []
            for hb in (0, 1):
                a = np.full((64, 32), one, np.uint8)
                b = np.zeros((64, 32), np.uint8)
                for col in range(32):
                    b[hb * 32 + col, col] = one
                sa = np.full(64, 127)
                sa[lane] = 128
                c = raw(fmt, a, b, sa, np.full(64, 127))
                for row, col in zip(*np.nonzero(c == 2.0)):
                    covered.append([int(row), hb, int(col)])  # (row, slot h, slot j)
            rows = sorted({x[0] for x in covered})
            cover[lane] = {"rows": rows, "slots": sorted({(x[1], x[2]) for x in covered})}
        res["a_scale_cover"] = {str(k): {"rows": v["rows"], "n_slots": len(v["slots"]),
                                         "slots": [list(s) for s in v["slots"]]} for k, v in cover.items()}
        out[fmt] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
