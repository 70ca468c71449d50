"""Generate tests/golden/ref_element_ops.json from the REFERENCE ITSELF.

The outputs are computed by the reference's own element operations,
reduce-op.c:71-150 (sum/prod, and/or/xor, min/max for every type it defines),
compiled from its text by oracle/build_ref.sh into oracle/_ref/libref_ops.so.
Inputs are special values (NaN payloads, signalling NaNs, +-0, +-inf,
subnormals, extremes; x87 pseudo-NaN/pseudo-inf/unnormal/pseudo-denormal
encodings for long double; Annex G inf/NaN mixes for complex) crossed with
each other, plus seeded random bit patterns.  For every valid (type, op) the
fixture holds op(a[i], b[i]) and op(b[i], a[i]) -- what PE 0 and PE 1 of a
2-PE reduction compute (reduce-op.c:213-248).

Run here (the GPU box has no /root/reference): python tests/golden/make_ref_ops.py
Test infrastructure only.
"""
import base64
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as O  # noqa: E402

REF_SO = os.path.join(REPO, "oracle", "_ref", "libref_ops.so")
OUT = os.path.join(HERE, "ref_element_ops.json")
NRAND = 256
TYPES = ["short", "int", "long", "longlong", "float", "double", "longdouble",
         "complexd", "complexf"]
OPS = ["sum", "prod", "and", "or", "xor", "min", "max"]


def ref_lib():
    L = ctypes.CDLL(REF_SO)
    vp = ctypes.c_void_p
    L.ref_op_apply.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, vp, ctypes.c_long]
    L.ref_op_apply.restype = ctypes.c_int
    return L


def ref_apply(L, t, op, a, b):
    out = np.zeros_like(a)
    rc = L.ref_op_apply(O.TYPES[t], O.OPS[op], a.ctypes.data, b.ctypes.data,
                        out.ctypes.data, a.size)
    return out if rc == 0 else None


def _rand_words(seed, n):
    return O.splitmix64(seed, n)


def _fp_specials(bits):
    ft = np.float32 if bits == 32 else np.float64
    ut = np.uint32 if bits == 32 else np.uint64
    fi = np.finfo(ft)
    vals = np.array([0.0, -0.0, np.inf, -np.inf, 1.0, -1.0, 2.5, -3.0, fi.tiny, -fi.tiny,
                     fi.tiny / 4, -fi.tiny / 8, fi.max, -fi.max, fi.eps, 1 + fi.eps,
                     np.sqrt(fi.max) * 2, fi.tiny * 3], dtype=ft)
    if bits == 64:
        nans = np.array([0x7FF8000000000000, 0xFFF8000000000000, 0x7FF0000000000001,
                         0x7FFC00000000BEEF, 0xFFF4000000001234], dtype=ut).view(ft)
    else:
        nans = np.array([0x7FC00000, 0xFFC00000, 0x7F800001, 0x7FE0BEEF, 0xFFA01234],
                        dtype=ut).view(ft)
    return np.concatenate([vals, nans])


def _ld_from_parts(sign_exp, mant):
    """x87 80-bit encodings in 16-byte slots (padding zero)."""
    n = len(mant)
    raw = np.zeros((n, 16), np.uint8)
    raw[:, 0:8] = np.array(mant, dtype=np.uint64).view(np.uint8).reshape(n, 8)
    raw[:, 8:10] = np.array(sign_exp, dtype=np.uint16).view(np.uint8).reshape(n, 2)
    return raw.view(np.longdouble).reshape(n)


def _ld_specials():
    J = 1 << 63
    se = [0x0000, 0x8000, 0x7FFF, 0xFFFF, 0x3FFF, 0xBFFF, 0x4000, 0x0001, 0x8001,
          0x0000, 0x7FFE, 0xFFFE,
          0x7FFF, 0x7FFF, 0xFFFF, 0x7FFF,      # NaNs: quiet, signalling, -quiet, payload
          0x7FFF, 0x7FFF,                      # pseudo-NaN, pseudo-inf (J bit clear)
          0x3FFF, 0x0000]                      # unnormal, pseudo-denormal
    m = [0, 0, J, J, J, J, J | (1 << 62), J, J,
         0x0000000000000F00, 0xFFFFFFFFFFFFFFFF, 0xFFFFFFFFFFFFFFFF,
         J | (1 << 62), J | 1, J | (1 << 62), J | (1 << 62) | 0xBEEF,
         (1 << 62) | 5, 0, 1 << 62, J | 7]
    return _ld_from_parts(se, m)


def _ld_random(seed, n):
    w = _rand_words(seed, 2 * n)
    mant = w[:n] | np.uint64(1 << 63)          # normal-looking significands
    exps = (w[n:] & np.uint64(0x7F)).astype(np.int64) - 64 + 0x3FFF
    sign = ((w[n:] >> np.uint64(8)) & np.uint64(1)).astype(np.int64) << 15
    # every 16th one a raw encoding (any J bit, any exponent)
    raw = (w[n:] >> np.uint64(16)) & np.uint64(0xFFFF)
    se = np.where(np.arange(n) % 16 == 0, raw.astype(np.int64), exps + sign)
    mant = np.where(np.arange(n) % 16 == 0, w[:n], mant)
    return _ld_from_parts(se.astype(np.uint16), mant)


def inputs(t):
    """(a, b): every special against every special, then NRAND random pairs."""
    dt = np.dtype(O.NP_DTYPE[t])
    seed = 0xE1E0 + O.TYPES[t]
    if t in ("short", "int", "long", "longlong"):
        info = np.iinfo(dt)
        s = np.array([info.min, info.max, 0, -1, 1, info.min + 1, info.max - 1, 12345, -777,
                      2], dtype=dt)
        r = _rand_words(seed, 2 * NRAND).view(np.uint64)
        ra = r[:NRAND].astype(f"u{dt.itemsize}").view(dt)
        rb = r[NRAND:].astype(f"u{dt.itemsize}").view(dt)
    elif t in ("float", "double"):
        bits = 8 * dt.itemsize
        s = _fp_specials(bits)
        ut = np.dtype(f"u{dt.itemsize}")
        r = _rand_words(seed, 2 * NRAND)
        half = NRAND // 2
        # half raw bit patterns, half values in [-4, 4) (products and sums that round)
        raw = r.astype(ut) if bits == 32 else r
        vals = ((r >> np.uint64(11)).astype(np.float64) * 2.0 ** -53 * 8 - 4).astype(dt)
        ra = np.concatenate([raw[:half].view(dt), vals[:NRAND - half]])
        rb = np.concatenate([raw[NRAND:NRAND + half].view(dt), vals[NRAND + half:]])
    elif t == "longdouble":
        s = _ld_specials()
        ra = _ld_random(seed, NRAND)
        rb = _ld_random(seed + 1, NRAND)
    else:
        ft = np.float64 if t == "complexd" else np.float32
        c = np.array([0.0, -0.0, -2.5, np.inf, -np.inf, np.nan], dtype=ft)
        re, im = np.meshgrid(c, c, indexing="ij")
        s = np.zeros(re.size, dt)
        sv = s.view(ft).reshape(-1, 2)
        sv[:, 0], sv[:, 1] = re.ravel(), im.ravel()
        r = _rand_words(seed, 4 * NRAND)
        v = ((r >> np.uint64(11)).astype(np.float64) * 2.0 ** -53 * 8 - 4).astype(ft)
        ra = v[:2 * NRAND].view(dt)
        rb = v[2 * NRAND:].view(dt)
    sa, sb = np.meshgrid(np.arange(len(s)), np.arange(len(s)), indexing="ij")
    a = np.concatenate([s[sa.ravel()], ra]).astype(dt)
    b = np.concatenate([s[sb.ravel()], rb]).astype(dt)
    return np.ascontiguousarray(a), np.ascontiguousarray(b)


def enc(x):
    return base64.b64encode(np.ascontiguousarray(x).tobytes()).decode()


def dec(s, t):
    return np.frombuffer(base64.b64decode(s), dtype=O.NP_DTYPE[t]).copy()


def main():
    L = ref_lib()
    out = {"source": "reduce-op.c:71-150 compiled from the reference's own text "
                     "(oracle/build_ref.sh, gcc -std=c99, no -O: configure's defaults)",
           "cases": {}}
    for t in TYPES:
        a, b = inputs(t)
        entry = {"a": enc(a), "b": enc(b), "ops": {}}
        for op in OPS:
            ab = ref_apply(L, t, op, a, b)
            if ab is None:
                assert not O.op_valid(t, op), (t, op)
                continue
            assert O.op_valid(t, op), (t, op)
            entry["ops"][op] = {"ab": enc(ab), "ba": enc(ref_apply(L, t, op, b, a))}
        out["cases"][t] = entry
    with open(OUT, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
