"""Checkpoint loader (wfamd/loader.py): the golden 2-layer model written to disk
in the three forms the reference handles -- HF packed uint8 [N/4, K] + weight_scale
(tests/test_bitnet_core.py:21-53), the reference's converted cache (`*.qweight` blocked I2_S,
cache/bitnet_converter.py:103-187, format packed_bitnet_v1) and float ternary `*.weight` -- loads
to the same I2_S bytes and decodes the reference's golden logits. Parsing/naming runs on CPU; the
repacking kernels and the decode step run on the GPU."""
import json

import numpy as np
import pytest
import torch

from conftest import load_golden

NAMES = (("wq", "self_attn.q_proj"), ("wk", "self_attn.k_proj"), ("wv", "self_attn.v_proj"),
         ("wo", "self_attn.o_proj"), ("wg", "mlp.gate_proj"), ("wu", "mlp.up_proj"), ("wd", "mlp.down_proj"))
NORMS = (("ln_in", "input_layernorm"), ("ln_post", "post_attention_layernorm"),
         ("attn_sub", "self_attn.attn_sub_norm"), ("ffn_sub", "mlp.ffn_sub_norm"))


def _bf16(bits: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(bits.astype(np.int16)).view(torch.bfloat16)


def _hf_pack(tern: np.ndarray) -> np.ndarray:
    """Inverse of the HF unpack (tests/test_bitnet_core.py:21-53): row i*(N/4)+r -> bits 2i of row r."""
    n, k = tern.shape
    q = n // 4
    enc = (tern + 1).astype(np.uint8).reshape(4, q, k)
    return (enc[0] | enc[1] << 2 | enc[2] << 4 | enc[3] << 6).astype(np.uint8)


def write_checkpoint(path, g: dict, form: str) -> None:
    """The golden decode model as a checkpoint directory in `form` in {'hf', 'cache', 'float'}."""
    from safetensors.torch import save_file

    from oracle import oracle as orc
    H, L, HQ, HKV, D, I, V, S = (int(v) for v in g["cfg"])
    cfg = {"hidden_size": H, "num_hidden_layers": L, "num_attention_heads": HQ, "num_key_value_heads": HKV,
           "intermediate_size": I, "vocab_size": V, "rms_norm_eps": float(g["eps"]), "rope_theta": 500000.0,
           "tie_word_embeddings": True}
    (path / "config.json").write_text(json.dumps(cfg))
    t = {"model.embed_tokens.weight": _bf16(g["embed"]), "model.norm.weight": _bf16(g["final_norm"])}
    for l in range(L):
        pre = f"model.layers.{l}"
        for key, sub in NORMS:
            t[f"{pre}.{sub}.weight"] = _bf16(g[key][l])
        for j, (key, sub) in enumerate(NAMES):
            i2s = g[key][l]
            k = i2s.shape[1] * 4
            ws = torch.tensor([float(g["wscale"][l, j])], dtype=torch.bfloat16 if form == "hf" else torch.float32)
            if form == "cache":
                t[f"{pre}.{sub}.qweight"] = torch.from_numpy(np.ascontiguousarray(i2s))
            else:
                tern = orc.unpack_i2s(i2s, k)
                if form == "hf":
                    t[f"{pre}.{sub}.weight"] = torch.from_numpy(_hf_pack(tern.astype(np.int8)))
                else:
                    t[f"{pre}.{sub}.weight"] = torch.from_numpy(tern).to(torch.bfloat16)
            t[f"{pre}.{sub}.weight_scale"] = ws
    half = len(t) // 2  # two shards, like a multi-file checkpoint
    keys = sorted(t)
    save_file({k: t[k].contiguous() for k in keys[:half]}, str(path / "model-00001-of-00002.safetensors"))
    save_file({k: t[k].contiguous() for k in keys[half:]}, str(path / "model-00002-of-00002.safetensors"))
    if form == "cache":
        (path / "cache_metadata.json").write_text(json.dumps({"format_version": "packed_bitnet_v1"}))


def test_config_and_format_detection(tmp_path):
    from wfamd import loader
    g = load_golden("decode")
    write_checkpoint(tmp_path, g, "cache")
    assert loader.checkpoint_format(tmp_path) == "packed_bitnet_v1"
    cfg = loader.config_from_hf(json.loads((tmp_path / "config.json").read_text()), max_seq=64)
    H, L, HQ, HKV, D, I, V, S = (int(v) for v in g["cfg"])
    assert (cfg.hidden, cfg.layers, cfg.n_heads, cfg.n_kv_heads, cfg.head_dim, cfg.inter, cfg.vocab) == \
        (H, L, HQ, HKV, D, I, V)
    t = loader._Tensors(tmp_path)
    assert "model.layers.1.mlp.down_proj.qweight" in t and len(t.names()) == 2 + L * (4 + 14)
    two_b = loader.config_from_hf({"hidden_size": 2560, "num_hidden_layers": 30, "num_attention_heads": 20,
                                   "num_key_value_heads": 5, "intermediate_size": 6912, "vocab_size": 128256})
    assert two_b == loader.BitNetConfig()


@pytest.mark.gpu
@pytest.mark.parametrize("form", ["hf", "cache", "float"])
def test_load_forms_decode_golden(tmp_path, form):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from oracle import oracle as orc
    from wfamd import loader
    from wfamd.model import BitNetDecoder, weights_from_arrays
    g = load_golden("decode")
    write_checkpoint(tmp_path, g, form)
    cfg, w = loader.load_checkpoint(tmp_path, max_seq=int(g["cfg"][7]))
    ref_w = weights_from_arrays(g)
    for key, _ in NAMES:
        assert torch.equal(w[key], ref_w[key]), (form, key)
    ws_ref = ref_w["wscale"] if form != "hf" else ref_w["wscale"].to(torch.bfloat16).float()
    assert torch.equal(w["wscale"], ws_ref)
    if form != "hf":  # the HF form stores the scale as bf16 (the checkpoint's dtype); the golden's is fp32
        dec = BitNetDecoder(cfg, w, batch=1)
        for step, tok in enumerate(g["tokens"][:3]):
            dec.set_state([int(tok)], [step])
            dec.step(graph=False)
            torch.cuda.synchronize()
            got = orc.bf16_to_f32(dec.logits[0].view(torch.int16).cpu().numpy().view(np.uint16))
            ref = orc.bf16_to_f32(g["logits"][step])
            assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < 1e-3, (form, step)
