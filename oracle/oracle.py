"""numpy front-end of the CPU ORACLE (liborc.so) -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, always as the
checker. The product package (wrinklefree-inference-engine_amd/) never imports this module.
Semantics and reference citations live in wf_oracle.c next to each function.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_lib = None


def build(march: str | None = None, name: str = "liborc.so", defines=()) -> Path:
    """liborc.so = the checker (make); any other name = a CPU-baseline build for this host
    (-march=native; defines=("ORC_VNNI",) for the AVX512-VNNI / BF16 kernels)."""
    args = ["make", "-s", "-C", str(_HERE), name] if name == "liborc.so" else None
    if name == "liborc.so":
        if march:
            args.append(f"MARCH={march}")
        subprocess.run(args, check=True)
    else:  # a separately named build (e.g. -march=native for the CPU baseline on the GPU box's host)
        out = _HERE / name
        subprocess.run(["gcc", "-O3", f"-march={march or 'native'}", "-fopenmp", "-fPIC", "-std=c11", "-shared"] +
                       [f"-D{d}" for d in defines] + ["-o", str(out), str(_HERE / "wf_oracle.c"), "-lm"], check=True)
    return _HERE / name


def lib(name: str = "liborc.so"):
    global _lib
    if name != "liborc.so":
        return _load(_HERE / name)
    if _lib is None:
        path = _HERE / name
        if not path.exists():
            build()
        _lib = _load(path)
    return _lib


def _load(path: Path):
    L = C.CDLL(str(path))
    vp, i32, i64, f32 = C.c_void_p, C.c_int, C.c_int64, C.c_float
    sig = {
        "orc_rmsnorm_bf16": [vp, vp, i32, f32, vp],
        "orc_pack_i2s": [vp, i32, i32, vp], "orc_unpack_i2s": [vp, i32, i32, vp],
        "orc_unpack_hf": [vp, i32, i32, vp], "orc_pack_lsb": [vp, i32, i32, vp],
        "orc_unpack_lsb": [vp, i32, i32, vp], "orc_pack_tq": [vp, i32, i32, vp],
        "orc_unpack_tq": [vp, i32, i32, vp],
        "orc_quantize_i8": [vp, i64, vp, vp], "orc_quantize_i8_rows": [vp, i32, i32, vp, vp],
        "orc_quantize_i8_trunc": [vp, i64, vp, vp],
        "orc_gemv_i2s": [vp, vp, f32, i32, i32, vp], "orc_gemm_i2s": [vp, vp, f32, i32, i32, i32, vp],
        "orc_gemv_lsb_signed": [vp, vp, f32, i32, i32, vp], "orc_enc_sums_i2s": [vp, vp, i32, i32, i32, vp],
        "orc_bitnet_linear_bf16": [vp, vp, f32, i32, i32, vp],
        "orc_attention_gqa_bf16": [vp, vp, vp, i32, i32, i32, i32, i32, f32, vp],
        "orc_attention_gqa_f32": [vp, vp, vp, i32, i32, i32, i32, i32, f32, vp],
        "orc_attention_sdpa_cpu_bf16": [vp, vp, vp, i32, i32, i32, i32, i32, vp],
        "orc_attention_sdpa_cpu_f32": [vp, vp, vp, i32, i32, i32, i32, i32, vp],
        "orc_decode_step": [vp, i32, i32, vp, vp],
        "orc_msb_ternarize": [vp, i32, i32, i32, f32, vp], "orc_msb_dequant": [vp, i32, i32, f32, vp],
        "orc_msb_linear": [vp, f32, vp, vp, i32, i32, i32, i32, vp],
    }
    for name, argt in sig.items():
        fn = getattr(L, name)
        fn.argtypes = argt
        fn.restype = C.c_int
    L.orc_tq_row_bytes.argtypes = [i32]
    L.orc_tq_row_bytes.restype = i64
    L.orc_f32_to_e4m3.argtypes = [f32]
    L.orc_f32_to_e4m3.restype = C.c_uint8
    L.orc_e4m3_to_f32.argtypes = [C.c_uint8]
    L.orc_e4m3_to_f32.restype = f32
    L.orc_fexp_u20.argtypes = [f32]
    L.orc_fexp_u20.restype = f32
    L.orc_vnni_build.argtypes = []
    L.orc_vnni_build.restype = C.c_int
    L.orc_num_threads.argtypes = []
    L.orc_num_threads.restype = C.c_int
    return L


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def _ck(rc: int, what: str):
    if rc != 0:
        raise ValueError(f"oracle {what} rejected its arguments (rc={rc})")


def pack_i2s(w: np.ndarray) -> np.ndarray:
    w = np.ascontiguousarray(w, dtype=np.float32)
    n, k = w.shape
    out = np.zeros((n, k // 4), np.uint8)
    _ck(lib().orc_pack_i2s(_p(w), n, k, _p(out)), "pack_i2s")
    return out


def unpack_i2s(p: np.ndarray, k: int) -> np.ndarray:
    p = np.ascontiguousarray(p, dtype=np.uint8)
    out = np.zeros((p.shape[0], k), np.float32)
    _ck(lib().orc_unpack_i2s(_p(p), p.shape[0], k, _p(out)), "unpack_i2s")
    return out


def unpack_hf(p: np.ndarray) -> np.ndarray:
    p = np.ascontiguousarray(p, dtype=np.uint8)
    out = np.zeros((p.shape[0] * 4, p.shape[1]), np.float32)
    _ck(lib().orc_unpack_hf(_p(p), p.shape[0], p.shape[1], _p(out)), "unpack_hf")
    return out


def pack_lsb(w: np.ndarray) -> np.ndarray:
    w = np.ascontiguousarray(w, dtype=np.float32)
    out = np.zeros((w.shape[0], w.shape[1] // 4), np.uint8)
    _ck(lib().orc_pack_lsb(_p(w), w.shape[0], w.shape[1], _p(out)), "pack_lsb")
    return out


def unpack_lsb(p: np.ndarray) -> np.ndarray:
    p = np.ascontiguousarray(p, dtype=np.uint8)
    out = np.zeros((p.shape[0], p.shape[1] * 4), np.float32)
    _ck(lib().orc_unpack_lsb(_p(p), p.shape[0], p.shape[1] * 4, _p(out)), "unpack_lsb")
    return out


def tq_row_bytes(k: int) -> int:
    return int(lib().orc_tq_row_bytes(k))


def pack_tq(i2s: np.ndarray) -> np.ndarray:
    i2s = np.ascontiguousarray(i2s, dtype=np.uint8)
    n, k = i2s.shape[0], i2s.shape[1] * 4
    out = np.zeros((n, tq_row_bytes(k)), np.uint8)
    _ck(lib().orc_pack_tq(_p(i2s), n, k, _p(out)), "pack_tq")
    return out


def unpack_tq(tq: np.ndarray, k: int) -> np.ndarray:
    tq = np.ascontiguousarray(tq, dtype=np.uint8)
    out = np.zeros((tq.shape[0], k // 4), np.uint8)
    _ck(lib().orc_unpack_tq(_p(tq), tq.shape[0], k, _p(out)), "unpack_tq")
    return out


def quantize_i8(x: np.ndarray):
    x = np.ascontiguousarray(x, dtype=np.float32)
    q = np.zeros(x.shape, np.int8)
    s = C.c_double()
    _ck(lib().orc_quantize_i8(_p(x), x.size, _p(q), C.addressof(s)), "quantize_i8")
    return q, s.value


def quantize_i8_rows(x: np.ndarray):
    x = np.ascontiguousarray(x, dtype=np.float32)
    m, k = x.shape
    q = np.zeros(x.shape, np.int8)
    s = np.zeros(m, np.float64)
    _ck(lib().orc_quantize_i8_rows(_p(x), m, k, _p(q), _p(s)), "quantize_i8_rows")
    return q, s


def quantize_i8_trunc(x: np.ndarray):
    x = np.ascontiguousarray(x, dtype=np.float32)
    q = np.zeros(x.shape, np.int8)
    s = C.c_float()
    _ck(lib().orc_quantize_i8_trunc(_p(x), x.size, _p(q), C.addressof(s)), "quantize_i8_trunc")
    return q, s.value


def gemm_i2s(p: np.ndarray, a: np.ndarray, scale: float) -> np.ndarray:
    p = np.ascontiguousarray(p, dtype=np.uint8)
    a2 = np.ascontiguousarray(a.reshape(-1, a.shape[-1]), dtype=np.int8)
    m, k = a2.shape
    n = p.shape[0]
    y = np.zeros((m, n), np.float32)
    _ck(lib().orc_gemm_i2s(_p(p), _p(a2), float(scale), m, n, k, _p(y)), "gemm_i2s")
    return y.reshape(*a.shape[:-1], n)


def gemv_i2s(p, a, scale):
    return gemm_i2s(p, a, scale)


def enc_sums_i2s(p: np.ndarray, a: np.ndarray) -> np.ndarray:
    p = np.ascontiguousarray(p, dtype=np.uint8)
    a2 = np.ascontiguousarray(a.reshape(-1, a.shape[-1]), dtype=np.int8)
    m, k = a2.shape
    s = np.zeros((m, p.shape[0]), np.int32)
    _ck(lib().orc_enc_sums_i2s(_p(p), _p(a2), m, p.shape[0], k, _p(s)), "enc_sums_i2s")
    return s


def gemv_lsb_signed(p: np.ndarray, a: np.ndarray, scale: float) -> np.ndarray:
    p = np.ascontiguousarray(p, dtype=np.uint8)
    a = np.ascontiguousarray(a, dtype=np.int8)
    y = np.zeros(p.shape[0], np.float32)
    _ck(lib().orc_gemv_lsb_signed(_p(p), _p(a), float(scale), p.shape[0], a.shape[0], _p(y)), "gemv_lsb")
    return y


def bitnet_linear_bf16(x_bits: np.ndarray, p: np.ndarray, ws: float) -> np.ndarray:
    x_bits = np.ascontiguousarray(x_bits, dtype=np.uint16)
    p = np.ascontiguousarray(p, dtype=np.uint8)
    y = np.zeros(p.shape[0], np.uint16)
    _ck(lib().orc_bitnet_linear_bf16(_p(x_bits), _p(p), float(ws), p.shape[0], x_bits.shape[0], _p(y)), "linear")
    return y


def rms_norm_bf16(x_bits: np.ndarray, w_bits: np.ndarray, eps: float) -> np.ndarray:
    """rms_norm of one bf16 row (scripts/direct_inference_full.py:181-184; the decode step's norm)."""
    x_bits = np.ascontiguousarray(x_bits, dtype=np.uint16)
    w_bits = np.ascontiguousarray(w_bits, dtype=np.uint16)
    y = np.zeros(x_bits.shape[0], np.uint16)
    _ck(lib().orc_rmsnorm_bf16(_p(x_bits), _p(w_bits), x_bits.shape[0], float(eps), _p(y)), "rmsnorm")
    return y


def attention_gqa_bf16(q_bits, k_bits, v_bits, s: int, scale: float | None = None) -> np.ndarray:
    """q [Hq, D]; k/v [Hkv, S_max, D] (bf16 bit patterns)."""
    q_bits = np.ascontiguousarray(q_bits, dtype=np.uint16)
    k_bits = np.ascontiguousarray(k_bits, dtype=np.uint16)
    v_bits = np.ascontiguousarray(v_bits, dtype=np.uint16)
    hq, d = q_bits.shape
    hkv, smax, _ = k_bits.shape
    out = np.zeros((hq, d), np.uint16)
    sc = float(scale) if scale is not None else 1.0 / float(np.sqrt(np.float32(d)))
    _ck(lib().orc_attention_gqa_bf16(_p(q_bits), _p(k_bits), _p(v_bits), hq, hkv, d, smax, s, sc, _p(out)), "attn")
    return out


def attention_gqa_f32(q_bits, k_bits, v_bits, s: int, scale: float | None = None) -> np.ndarray:
    """attention_gqa_bf16 with the double result rounded to float32 (kernel-level attention check)."""
    q_bits = np.ascontiguousarray(q_bits, dtype=np.uint16)
    k_bits = np.ascontiguousarray(k_bits, dtype=np.uint16)
    v_bits = np.ascontiguousarray(v_bits, dtype=np.uint16)
    hq, d = q_bits.shape
    hkv, smax, _ = k_bits.shape
    out = np.zeros((hq, d), np.float32)
    sc = float(scale) if scale is not None else 1.0 / float(np.sqrt(np.float32(d)))
    _ck(lib().orc_attention_gqa_f32(_p(q_bits), _p(k_bits), _p(v_bits), hq, hkv, d, smax, s, sc, _p(out)), "attn32")
    return out


def attention_sdpa_cpu_bf16(q_bits, k_bits, v_bits, s: int) -> np.ndarray:
    """The reference's SDPA call as torch's CPU flash kernel computes it on bf16 (wf_oracle.c
    orc_attention_sdpa_cpu_bf16). q [Hq, D]; k/v [Hkv, S_max, D] (bf16 bit patterns)."""
    q_bits = np.ascontiguousarray(q_bits, dtype=np.uint16)
    k_bits = np.ascontiguousarray(k_bits, dtype=np.uint16)
    v_bits = np.ascontiguousarray(v_bits, dtype=np.uint16)
    hq, d = q_bits.shape
    hkv, smax, _ = k_bits.shape
    out = np.zeros((hq, d), np.uint16)
    _ck(lib().orc_attention_sdpa_cpu_bf16(_p(q_bits), _p(k_bits), _p(v_bits), hq, hkv, d, smax, s, _p(out)), "sdpa")
    return out


def attention_sdpa_cpu_f32(q_bits, k_bits, v_bits, s: int) -> np.ndarray:
    """attention_sdpa_cpu_bf16 before the output's bf16 rounding (float32 [Hq, D])."""
    q_bits = np.ascontiguousarray(q_bits, dtype=np.uint16)
    k_bits = np.ascontiguousarray(k_bits, dtype=np.uint16)
    v_bits = np.ascontiguousarray(v_bits, dtype=np.uint16)
    hq, d = q_bits.shape
    hkv, smax, _ = k_bits.shape
    out = np.zeros((hq, d), np.float32)
    _ck(lib().orc_attention_sdpa_cpu_f32(_p(q_bits), _p(k_bits), _p(v_bits), hq, hkv, d, smax, s, _p(out)), "sdpa32")
    return out


def fexp_u20(x: np.ndarray) -> np.ndarray:
    """torch's Vectorized<float>::fexp_u20, element-wise (the oracle's restatement)."""
    f = lib().orc_fexp_u20
    return np.array([f(float(v)) for v in np.asarray(x, np.float32).ravel()], np.float32).reshape(np.shape(x))


def e4m3_decode_table() -> np.ndarray:
    """float32 value of every OCP e4m3fn code (the oracle's decoder)."""
    return np.array([lib().orc_e4m3_to_f32(c) for c in range(256)], dtype=np.float32)


def int8_codes_to_bf16(codes: np.ndarray, scale: float) -> np.ndarray:
    """bf16 bits of int8 code * scale (what the oracle's int8 K/V rows hold); codes as int8 or their
    uint8 bytes."""
    v = np.asarray(codes).astype(np.uint8).view(np.int8).astype(np.float32) * np.float32(scale)
    return f32_to_bf16(v.astype(np.float32))


def fp8_codes_to_bf16(codes: np.ndarray, scale: float) -> np.ndarray:
    """bf16 bits of e4m3 code * scale (what the oracle's FP8 K/V rows hold)."""
    v = e4m3_decode_table()[np.asarray(codes, dtype=np.uint8)] * np.float32(scale)
    return f32_to_bf16(v.astype(np.float32))


class _Model(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("hidden", "layers", "n_heads", "n_kv_heads", "head_dim", "inter", "vocab",
                                        "max_seq")] + [("eps", C.c_float)] + \
               [(n, C.c_void_p) for n in ("embed", "final_norm", "rope_cos", "rope_sin", "ln_in", "ln_post",
                                          "attn_sub", "ffn_sub", "wq", "wk", "wv", "wo", "wg", "wu", "wd", "wscale",
                                          "k_cache", "v_cache")] + \
               [("kv_fp8", C.c_int), ("kv_scale", C.c_void_p), ("attn_mode", C.c_int)]


class DecodeModel:
    """Holds a model's host arrays (dict of numpy arrays in the tests/golden/decode.npz layout) for
    orc_decode_step. K/V caches are [layers, n_kv_heads, max_seq, head_dim] bf16 bits."""

    def __init__(self, arrays: dict, libname: str = "liborc.so", kv_fp8=False, kv_scale=None, attn_mode: int = 0):
        """kv_fp8: False / 0 bf16 K/V rows, True / 1 e4m3 rows, 2 int8 rows (orc_model.kv_fp8).
        attn_mode: 0 exact softmax (fp32-SDPA form), 1 the reference's CPU bf16 SDPA (orc_model)."""
        H, L, HQ, HKV, D, I, V, S = (int(x) for x in arrays["cfg"])
        self.cfg = (H, L, HQ, HKV, D, I, V, S)
        self.a = {k: np.ascontiguousarray(v) for k, v in arrays.items()}
        self.k_cache = np.zeros((L, HKV, S, D), np.uint16)
        self.v_cache = np.zeros((L, HKV, S, D), np.uint16)
        self._lib = lib(libname)
        m = _Model()
        m.hidden, m.layers, m.n_heads, m.n_kv_heads, m.head_dim, m.inter, m.vocab, m.max_seq = H, L, HQ, HKV, D, I, V, S
        m.eps = float(arrays.get("eps", 1e-5))
        for n in ("embed", "final_norm", "rope_cos", "rope_sin", "ln_in", "ln_post", "attn_sub", "ffn_sub",
                  "wq", "wk", "wv", "wo", "wg", "wu", "wd", "wscale"):
            setattr(m, n, _p(self.a[n]))
        m.k_cache, m.v_cache = _p(self.k_cache), _p(self.v_cache)
        self.kv_scale = np.ones((L, 2), np.float32) if kv_scale is None else np.ascontiguousarray(
            np.broadcast_to(np.asarray(kv_scale, dtype=np.float32), (L, 2)))
        m.kv_fp8, m.kv_scale = int(kv_fp8), _p(self.kv_scale)
        m.attn_mode = int(attn_mode)
        self.m = m

    def step(self, token: int, pos: int, logits: bool = True):
        """One token; logits=False appends the K/V rows only (no LM head) and returns (None, -1)."""
        out = np.zeros(self.cfg[6], np.uint16) if logits else None
        nxt = C.c_int()
        _ck(self._lib.orc_decode_step(C.addressof(self.m), int(token), int(pos), _p(out) if logits else None,
                                      C.addressof(nxt)), "decode_step")
        return out, nxt.value


def num_threads(libname: str = "liborc.so") -> int:
    return int(lib(libname).orc_num_threads())


def bf16_to_f32(bits: np.ndarray) -> np.ndarray:
    return (np.asarray(bits, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


def f32_to_bf16(x: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    nan = np.isnan(np.asarray(x, dtype=np.float32))
    return np.where(nan, (u >> 16).astype(np.uint16) | 0x40, r).astype(np.uint16)


# ---- SGLang BitNet linear method, MSB-interleaved layout (§8 a12) ----
_MSB_DT = {"float32": 0, "bfloat16": 1, "float16": 2}


def msb_ternarize(w: np.ndarray, scale: float, dtype: str = "float32") -> np.ndarray:
    """w: float32 array holding values of `dtype`; returns uint8 [N, K/4]."""
    w = np.ascontiguousarray(w, dtype=np.float32)
    n, k = w.shape
    out = np.zeros((n, k // 4), np.uint8)
    _ck(lib().orc_msb_ternarize(_p(w), _MSB_DT[dtype], n, k, float(scale), _p(out)), "msb_ternarize")
    return out


def msb_dequant(p: np.ndarray, scale: float) -> np.ndarray:
    p = np.ascontiguousarray(p, dtype=np.uint8)
    out = np.zeros((p.shape[0], p.shape[1] * 4), np.float32)
    _ck(lib().orc_msb_dequant(_p(p), p.shape[0], p.shape[1] * 4, float(scale), _p(out)), "msb_dequant")
    return out


def msb_linear(p: np.ndarray, ws: float, x: np.ndarray, bias: np.ndarray | None = None,
               dtype: str = "bfloat16") -> np.ndarray:
    """x [M, K] float32 holding values of `dtype`; ws = the weight scale rounded to `dtype`."""
    p = np.ascontiguousarray(p, dtype=np.uint8)
    x = np.ascontiguousarray(x, dtype=np.float32)
    b = None if bias is None else np.ascontiguousarray(bias, dtype=np.float32)
    m, k = x.shape
    y = np.zeros((m, p.shape[0]), np.float32)
    _ck(lib().orc_msb_linear(_p(p), float(ws), _p(x), None if b is None else _p(b), _MSB_DT[dtype], m, p.shape[0],
                             k, _p(y)), "msb_linear")
    return y
