"""Frozen Gemma3 causal LM on libptk (`ptk_gemma3_loss_fwd_bwd`).

Replaces `language_model(inputs_embeds=, attention_mask=, labels=).loss`
followed by `accelerator.backward(...)` down to d(inputs_embeds)
(Stage1/projector_trainer.py:183-237 -> TF/models/gemma3/modeling_gemma3.py
:511-659, TF/loss/loss_utils.py:49-67).  The frozen weights get no grads, so
only the dX chain is computed.

Kernel layouts built once from HF-named weights: q|k|v fused rows, gate/up
interleaved in 16-row blocks (the GEGLU GEMM epilogue pairs them in
registers), and a pre-transposed copy of every matrix for the dX GEMMs.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib as L
from . import kernels as K
from .config import Gemma3TextConfig


def _dev(a, dtype, device):
    t = torch.from_numpy(a) if isinstance(a, np.ndarray) else a
    return t.to(device=device, dtype=dtype).contiguous()


def interleave_gate_up(gate, up):
    """[I,H],[I,H] -> [2I,H]: rows 32q..32q+15 = gate[16q..16q+15], 32q+16.. = up[16q..]."""
    I, H = gate.shape
    return torch.stack([gate.view(I // 16, 16, H), up.view(I // 16, 16, H)], dim=1).reshape(2 * I, H).contiguous()


def rope_tables(cfg: Gemma3TextConfig, max_pos: int, sliding: bool):
    """Gemma3RotaryEmbedding math (modeling_gemma3.py:156-205) in fp32 on the host:
    returns cos, sin [max_pos, head_dim/2] (emb = [f, f] so the second half repeats)."""
    d = cfg.head_dim
    theta = cfg.rope_local_base_freq if sliding else cfg.rope_theta
    inv = 1.0 / (theta ** (torch.arange(0, d, 2, dtype=torch.int64).float() / d))
    if not sliding and cfg.rope_linear_factor != 1.0:
        inv = inv / cfg.rope_linear_factor
    f = torch.arange(max_pos, dtype=torch.float32)[:, None] * inv[None, :]
    return f.cos().contiguous(), f.sin().contiguous()


class Gemma3CausalLM:
    def __init__(self, cfg: Gemma3TextConfig, params: dict | None, device="cuda", max_pos: int = 2048):
        self.cfg, self.device, self.max_pos = cfg, torch.device(device), max_pos
        self._ws = None
        if params is not None:
            self._load(params)
            self._build_c()

    # ------------------------------------------------------------------ weights
    def _load(self, params):
        cfg, dev = self.cfg, self.device
        bf, f32 = torch.bfloat16, torch.float32
        g = lambda n, dt: _dev(params[n], dt, dev)
        self.embed = g("model.embed_tokens.weight", bf)
        self.final_norm = g("model.norm.weight", f32)
        self.layers = []
        for i in range(cfg.num_hidden_layers):
            p = f"model.layers.{i}."
            wqkv = torch.cat([g(p + f"self_attn.{n}_proj.weight", bf) for n in "qkv"]).contiguous()
            wgu = interleave_gate_up(g(p + "mlp.gate_proj.weight", bf), g(p + "mlp.up_proj.weight", bf))
            lay = dict(wqkv=wqkv, wo=g(p + "self_attn.o_proj.weight", bf), wgu=wgu,
                       wd=g(p + "mlp.down_proj.weight", bf),
                       ln_in=g(p + "input_layernorm.weight", f32),
                       ln_post_attn=g(p + "post_attention_layernorm.weight", f32),
                       ln_pre_ff=g(p + "pre_feedforward_layernorm.weight", f32),
                       ln_post_ff=g(p + "post_feedforward_layernorm.weight", f32),
                       q_norm=g(p + "self_attn.q_norm.weight", f32), k_norm=g(p + "self_attn.k_norm.weight", f32))
            self.layers.append(lay)
        self._derive()

    def _derive(self):
        for lay in self.layers:
            for k in ("wqkv", "wo", "wgu", "wd"):
                lay[k + "_t"] = K.transpose(lay[k])
        self.embed_t = K.transpose(self.embed)
        tabs = [rope_tables(self.cfg, self.max_pos, s) for s in (True, False)]
        (self.cos_l, self.sin_l), (self.cos_g, self.sin_g) = [(c.to(self.device), s.to(self.device))
                                                              for c, s in tabs]

    @staticmethod
    def config_from_hf(c) -> Gemma3TextConfig:
        """Gemma3TextConfig from an HF config of either shape:
        * transformers 4.51 (the reference's pin, requirements.txt:6): `sliding_window_pattern`,
          `rope_theta`, `rope_local_base_freq`, `rope_scaling` ({"rope_type": "linear", "factor": f} or None);
        * transformers >= 5: `layer_types` and per-layer-type `rope_parameters`."""
        lt = getattr(c, "layer_types", None)
        rp = getattr(c, "rope_parameters", None)
        if lt is not None and isinstance(rp, dict) and "full_attention" in rp:
            lt = list(lt)
            pattern = lt.index("full_attention") + 1 if "full_attention" in lt else len(lt) + 1
            want = ["sliding_attention" if (i + 1) % pattern else "full_attention" for i in range(len(lt))]
            if lt != want:
                raise ValueError(f"Gemma3 layer_types {lt} are not a periodic sliding/full pattern")
            theta, local = rp["full_attention"]["rope_theta"], rp["sliding_attention"]["rope_theta"]
            factor = float(rp["full_attention"].get("factor", 1.0))
        else:
            pattern = int(c.sliding_window_pattern)
            theta, local = float(c.rope_theta), float(c.rope_local_base_freq)
            rs = getattr(c, "rope_scaling", None) or {}
            kind = rs.get("rope_type", rs.get("type", "default"))
            if kind not in ("default", "linear"):
                raise ValueError(f"Gemma3 rope_scaling type {kind!r} is not supported (default / linear only)")
            factor = float(rs.get("factor", 1.0)) if kind == "linear" else 1.0
        return Gemma3TextConfig(vocab_size=c.vocab_size, hidden_size=c.hidden_size,
                                intermediate_size=c.intermediate_size, num_hidden_layers=c.num_hidden_layers,
                                num_attention_heads=c.num_attention_heads, num_key_value_heads=c.num_key_value_heads,
                                head_dim=c.head_dim, sliding_window=c.sliding_window, sliding_window_pattern=pattern,
                                rope_theta=theta, rope_local_base_freq=local, rope_linear_factor=factor,
                                query_pre_attn_scalar=c.query_pre_attn_scalar, rms_norm_eps=c.rms_norm_eps,
                                pad_token_id=c.pad_token_id if c.pad_token_id is not None else 0)

    @staticmethod
    def check_not_quantized(model):
        """The reference's --enable_qlora path loads the LM in 4 bit with LoRA adapters
        (Stage1/train_projection_stage1.py:192-210); the HIP path runs bf16 GEMMs on dense weights."""
        qc = getattr(getattr(model, "config", None), "quantization_config", None)
        if (getattr(model, "is_loaded_in_4bit", False) or getattr(model, "is_loaded_in_8bit", False)
                or getattr(model, "is_quantized", False) or qc is not None or hasattr(model, "peft_config")):
            raise ValueError("Gemma3CausalLM.from_hf: quantised / QLoRA (peft) language models are not supported "
                             "by the HIP Stage-1 path; pass the dense bf16 or fp32 Gemma3ForCausalLM "
                             "(run without --enable_qlora)")

    @classmethod
    def from_hf(cls, model, device="cuda", max_pos=2048):
        cls.check_not_quantized(model)
        cfg = cls.config_from_hf(model.config)
        sd = {k: v.detach().float() for k, v in model.state_dict().items()}
        lm = cls(cfg, sd, device, max_pos)
        # generate() without explicit sampling arguments uses the checkpoint's generation_config, as HF does (the
        # public gemma-3-1b-it ships top_k 64, top_p 0.95)
        gc = getattr(model, "generation_config", None)
        if gc is not None:
            lm.generation_defaults = {k: getattr(gc, k) for k in ("top_k", "top_p", "temperature")
                                      if getattr(gc, k, None) is not None}
        return lm

    @classmethod
    def random_init(cls, cfg: Gemma3TextConfig, device="cuda", seed=1, max_pos=2048):
        """Synthetic bf16 weights generated on the device (N(0, 0.02^2); norm weights 0)."""
        self = cls(cfg, None, device, max_pos)
        dev = self.device
        H, I = cfg.hidden_size, cfg.intermediate_size
        s = [seed * 100000]

        def nb(*shape, std=0.02):
            s[0] += 1
            return K.fill_normal_(torch.empty(shape, dtype=torch.bfloat16, device=dev), s[0], std)
        z = lambda n: torch.zeros(n, dtype=torch.float32, device=dev)
        self.embed = nb(cfg.vocab_size, H)
        self.final_norm = z(H)
        self.layers = [dict(wqkv=nb(cfg.q_dim + 2 * cfg.kv_dim, H), wo=nb(H, cfg.q_dim), wgu=nb(2 * I, H),
                            wd=nb(H, I), ln_in=z(H), ln_post_attn=z(H), ln_pre_ff=z(H), ln_post_ff=z(H),
                            q_norm=z(cfg.head_dim), k_norm=z(cfg.head_dim))
                       for _ in range(cfg.num_hidden_layers)]
        self._derive()
        self._build_c()
        return self

    def _build_c(self):
        c = self.cfg
        self.c_cfg = L.Gemma3ConfigC(c.vocab_size, c.hidden_size, c.intermediate_size, c.num_hidden_layers,
                                     c.num_attention_heads, c.num_key_value_heads, c.head_dim, c.sliding_window,
                                     c.sliding_window_pattern, c.pad_token_id, float(c.query_pre_attn_scalar),
                                     c.rms_norm_eps)
        keys = ("wqkv", "wqkv_t", "wo", "wo_t", "wgu", "wgu_t", "wd", "wd_t", "ln_in", "ln_post_attn", "ln_pre_ff",
                "ln_post_ff", "q_norm", "k_norm")
        arr = (L.Gemma3LayerC * len(self.layers))()
        for i, lay in enumerate(self.layers):
            arr[i] = L.Gemma3LayerC(*[lay[k].data_ptr() for k in keys])
        self._c_layers = arr
        self.c_w = L.Gemma3WeightsC(self.embed.data_ptr(), self.embed_t.data_ptr(), self.final_norm.data_ptr(),
                                    self.cos_l.data_ptr(), self.sin_l.data_ptr(), self.cos_g.data_ptr(),
                                    self.sin_g.data_ptr(), self.max_pos, C.cast(arr, C.POINTER(L.Gemma3LayerC)))

    # ------------------------------------------------------------------ compute
    @staticmethod
    def seq_pad(seq_len: int) -> int:
        return (seq_len + 63) // 64 * 64

    def workspace(self, batch, text_len, seq_pad):
        n = L.lib().ptk_gemma3_workspace_bytes(self.c_cfg, batch, text_len, seq_pad)
        if self._ws is None or self._ws.numel() < n:
            self._ws = None
            self._ws = torch.empty(n, dtype=torch.uint8, device=self.device)
        return self._ws

    def loss_and_input_grad(self, x, dx, token_ids, labels, num_vision, loss_scale, loss, pad_token_id=None):
        """x: f32 [B*Spad, H] LLM input rows (vision rows filled by the caller),
        token_ids/labels int64 [B, T].  Writes loss [1] (mean CE) and dx (grad of
        loss*loss_scale w.r.t. x; dx None = forward and loss only, ptk_gemma3_loss_fwd).  pad_token_id: id whose text positions are
        masked as keys (the trainer passes the tokenizer's, projector_trainer.py:207;
        -1 masks none); None = the model config's."""
        B, T = token_ids.shape
        Sp = x.shape[0] // B
        ws = self.workspace(B, T, Sp)
        bt = L.Gemma3BatchC(B, T, num_vision, Sp, token_ids.data_ptr(), labels.data_ptr(), x.data_ptr(),
                            0 if dx is None else dx.data_ptr(), loss_scale, loss.data_ptr())
        cfg = self.c_cfg
        if pad_token_id is not None and pad_token_id != cfg.pad_token_id:
            cfg = L.Gemma3ConfigC.from_buffer_copy(cfg)
            cfg.pad_token_id = int(pad_token_id)
        fn = "ptk_gemma3_loss_fwd" if dx is None else "ptk_gemma3_loss_fwd_bwd"
        L.check(getattr(L.lib(), fn)(cfg, self.c_w, bt, ws.data_ptr(), ws.numel(), L.stream_ptr(self.device)), fn)

    def get_input_embeddings(self):
        return self.embed

    generation_defaults: dict = {}   # HF GenerationConfig defaults unless the checkpoint ships its own

    def generate(self, inputs_embeds, max_new_tokens=64, do_sample=True, top_k=None, temperature=None,
                 pad_token_id=None, eos_token_id=None, seed=0, prompt_len=None, batch=None, force_ids=None,
                 return_logits=False, top_p=None):
        """`Gemma3ForCausalLM.generate(inputs_embeds=, attention_mask=ones, max_new_tokens=, do_sample=, pad_token_id=,
        eos_token_id=)` as the reference's validation calls it (Stage1/projector_trainer.py:386-393) on the KV-cache
        decode of libptk (ptk_gemma3_generate): returns the NEW tokens, int64 [B, n], n = max_new_tokens or the step
        at which every row has produced eos_token_id (HF's stopping; finished rows are padded with pad_token_id).
        Sampling follows HF's processors with the checkpoint's generation config where from_hf found one, else
        GenerationConfig's defaults (temperature 1, top_k 50, top_p 1); explicit arguments win.  The drawn tokens
        are one draw of the same distribution, from a counter-based generator seeded by `seed`
        (torch.multinomial's stream is not reproduced).
        inputs_embeds: f32 [B, P, H], or [B * stride, H] rows with prompt_len = P and batch = B (the Stage-1
        engine's LLM input, whose vision rows start each stride-row sample).  force_ids (int64 [B, max_new_tokens]): teacher forcing
        (step t feeds force_ids[:, t-1]); return_logits: also the bf16 logits of every step [max_new_tokens, B, V]."""
        if inputs_embeds.dtype != torch.float32 or not inputs_embeds.is_cuda or not inputs_embeds.is_contiguous():
            raise L.PtkError("generate: inputs_embeds must be a contiguous f32 HIP tensor")
        H = self.cfg.hidden_size
        if inputs_embeds.dim() == 3:
            B, P, _ = inputs_embeds.shape
            stride = P
        else:
            if prompt_len is None or batch is None or inputs_embeds.shape[0] % batch:
                raise L.PtkError("generate: 2-D inputs_embeds need prompt_len and batch (rows = batch x stride)")
            P, B = int(prompt_len), int(batch)
            stride = inputs_embeds.shape[0] // B
        if inputs_embeds.shape[-1] != H:
            raise L.PtkError(f"generate: inputs_embeds width {inputs_embeds.shape[-1]} != hidden {H}")
        pad = self.cfg.pad_token_id if pad_token_id is None else int(pad_token_id)
        eos = -1 if eos_token_id is None else int(eos_token_id)
        dflt = self.generation_defaults
        top_k = dflt.get("top_k", 50) if top_k is None else top_k
        top_p = dflt.get("top_p", 1.0) if top_p is None else top_p
        temperature = dflt.get("temperature", 1.0) if temperature is None else temperature
        desc = L.Gemma3GenerateC(B, P, max_new_tokens, int(bool(do_sample)), int(top_k or 0), float(temperature),
                                 int(seed) & ((1 << 64) - 1), eos, pad, stride, float(top_p))
        n = L.lib().ptk_gemma3_generate_workspace_bytes(self.c_cfg, B, P, max_new_tokens)
        if getattr(self, "_gen_ws", None) is None or self._gen_ws.numel() < n:
            self._gen_ws = None
            self._gen_ws = torch.empty(n, dtype=torch.uint8, device=self.device)
        out = torch.empty((B, max_new_tokens), dtype=torch.int64, device=self.device)
        logits = (torch.empty((max_new_tokens, B, self.cfg.vocab_size), dtype=torch.bfloat16, device=self.device)
                  if return_logits else None)
        if force_ids is not None:
            force_ids = force_ids.to(device=self.device, dtype=torch.int64).contiguous()
            if tuple(force_ids.shape) != (B, max_new_tokens):
                raise L.PtkError(f"generate: force_ids must be [{B}, {max_new_tokens}]")
        L.check(L.lib().ptk_gemma3_generate(self.c_cfg, self.c_w, desc, inputs_embeds.data_ptr(),
                                            0 if force_ids is None else force_ids.data_ptr(), out.data_ptr(),
                                            0 if logits is None else logits.data_ptr(), self._gen_ws.data_ptr(),
                                            self._gen_ws.numel(), L.stream_ptr(self.device)), "ptk_gemma3_generate")
        n_out = max_new_tokens
        if eos >= 0:   # HF stops after the step at which the last unfinished row produced EOS
            done = (out == eos).cumsum(1) > 0
            all_done = done.all(0).nonzero()
            if all_done.numel():
                n_out = int(all_done[0]) + 1
        out = out[:, :n_out]
        return (out, logits) if return_logits else out

    # ------------------------------------------------------------------ beam search (stepwise decode)
    def decode_begin(self, inputs_embeds, attention_mask=None, repeat=1, max_new_tokens=512):
        """Prefill of the stepwise decode (ptk_gemma3_decode_prefill): prompts [B, P, H] f32 with an optional
        attention mask [B, P] (0 = padding: a masked key, and HF's position ids cumsum(mask) - 1), each prompt
        given to `repeat` consecutive rows.  Returns the first logits, bf16 [B * repeat, V]."""
        if inputs_embeds.dtype != torch.float32 or not inputs_embeds.is_cuda or inputs_embeds.dim() != 3:
            raise L.PtkError("decode: inputs_embeds must be an f32 HIP tensor [B, P, H]")
        x = inputs_embeds.contiguous()
        B, P, H = x.shape
        if H != self.cfg.hidden_size:
            raise L.PtkError(f"decode: inputs_embeds width {H} != hidden {self.cfg.hidden_size}")
        self._dec = L.Gemma3DecodeC(B * repeat, P, max_new_tokens, repeat, P)
        n = L.lib().ptk_gemma3_decode_workspace_bytes(self.c_cfg, self._dec)
        if getattr(self, "_dec_ws", None) is None or self._dec_ws.numel() < n:
            self._dec_ws = None
            self._dec_ws = torch.empty(n, dtype=torch.uint8, device=self.device)
        mask = None
        if attention_mask is not None:
            mask = attention_mask.to(device=self.device, dtype=torch.int32).contiguous()
            if tuple(mask.shape) != (B, P):
                raise L.PtkError(f"decode: attention_mask must be [{B}, {P}]")
        self._dec_x = x   # keep the prompt alive for the call
        logits = torch.empty((B * repeat, self.cfg.vocab_size), dtype=torch.bfloat16, device=self.device)
        L.check(L.lib().ptk_gemma3_decode_prefill(self.c_cfg, self.c_w, self._dec, x.data_ptr(),
                                                  0 if mask is None else mask.data_ptr(), P, logits.data_ptr(),
                                                  self._dec_ws.data_ptr(), self._dec_ws.numel(),
                                                  L.stream_ptr(self.device)), "ptk_gemma3_decode_prefill")
        return logits

    def decode_next(self, step, ids, src_rows=None):
        """Decode step `step` (1..max_new_tokens-1): every row appends ids[row] after taking the cache of row
        src_rows[row] (beam re-ordering; None keeps each row's own).  Returns the logits bf16 [rows, V]."""
        rows = self._dec.rows
        ids = ids.to(device=self.device, dtype=torch.int64).contiguous()
        src = None if src_rows is None else src_rows.to(device=self.device, dtype=torch.int32).contiguous()
        if ids.numel() != rows or (src is not None and src.numel() != rows):
            raise L.PtkError(f"decode: ids / src_rows must hold {rows} rows")
        logits = torch.empty((rows, self.cfg.vocab_size), dtype=torch.bfloat16, device=self.device)
        L.check(L.lib().ptk_gemma3_decode_step(self.c_cfg, self.c_w, self._dec, int(step), ids.data_ptr(),
                                               0 if src is None else src.data_ptr(), logits.data_ptr(),
                                               self._dec_ws.data_ptr(), self._dec_ws.numel(),
                                               L.stream_ptr(self.device)), "ptk_gemma3_decode_step")
        return logits

    def beam_candidates(self, logits, beam_scores, beams, n_cand, do_sample, top_k, top_p, temperature, seed, step,
                        min_tokens_to_keep):
        """ptk_beam_candidates over logits [B * beams, V]: (tokens int64, beam int32, accumulated f32) [B, n_cand]."""
        rows, V = logits.shape
        B = rows // beams
        tok = torch.empty((B, n_cand), dtype=torch.int64, device=self.device)
        bi = torch.empty((B, n_cand), dtype=torch.int32, device=self.device)
        sc = torch.empty((B, n_cand), dtype=torch.float32, device=self.device)
        bs = beam_scores.to(device=self.device, dtype=torch.float32).contiguous()
        n = L.lib().ptk_beam_candidates_workspace_bytes(B, beams, n_cand)
        if getattr(self, "_bc_ws", None) is None or self._bc_ws.numel() < n:
            self._bc_ws = torch.empty(n, dtype=torch.uint8, device=self.device)
        L.check(L.lib().ptk_beam_candidates(logits.data_ptr(), V, bs.data_ptr(), B, beams, V, int(bool(do_sample)),
                                            int(top_k or 0), float(top_p), float(temperature), int(min_tokens_to_keep),
                                            int(seed) & ((1 << 64) - 1), int(step), int(n_cand), tok.data_ptr(),
                                            bi.data_ptr(), sc.data_ptr(), self._bc_ws.data_ptr(), self._bc_ws.numel(),
                                            L.stream_ptr(self.device)), "ptk_beam_candidates")
        return tok, bi, sc

    def beam_generate(self, inputs_embeds, attention_mask=None, num_beams=3, max_new_tokens=512, do_sample=True,
                      top_k=50, top_p=1.0, temperature=1.0, eos_token_id=None, pad_token_id=None,
                      length_penalty=1.0, early_stopping=False, seed=0):
        """`generate(inputs_embeds=, attention_mask=, num_beams=, do_sample=, top_k=, top_p=, ...)` with beams, as
        Stage 2's validation calls it (Stage2/trainer.py:596-626 -> GenerationMixin._beam_search): the stepwise
        KV-cache decode, ptk_beam_candidates for the continuations of each step (sampled without replacement from
        the joint beam x vocab distribution, or the best with do_sample=False) and the host bookkeeping of
        projectiontrainer_amd/beam.py.  Returns the new tokens of the best hypothesis per prompt, int64 [B, n]."""
        from .beam import BeamSearch
        B = inputs_embeds.shape[0]
        K = int(num_beams)
        n_eos = 0 if eos_token_id is None else 1
        n_cand = max(2, 1 + n_eos) * K
        min_keep = (1 + n_eos) if K > 1 else 1
        pad = self.cfg.pad_token_id if pad_token_id is None else int(pad_token_id)
        bs = BeamSearch(B, K, max_new_tokens, eos_token_id, pad, length_penalty, early_stopping)
        logits = self.decode_begin(inputs_embeds, attention_mask, repeat=K, max_new_tokens=max_new_tokens)
        step = 0
        while True:
            tok, bi, sc = self.beam_candidates(logits, bs.run_score.reshape(-1), K, n_cand, do_sample, top_k, top_p,
                                               temperature, seed, step, min_keep)
            ids, rows = bs.step(tok, bi, sc)
            if bs.finished:
                break
            step += 1
            logits = self.decode_next(step, ids, rows)
        return bs.result().to(self.device)
