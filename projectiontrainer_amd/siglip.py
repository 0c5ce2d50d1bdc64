"""Frozen SigLIP vision tower on libptk (`ptk_siglip_fwd`).

Replaces the reference's `vision_tower(pixel_values=...).last_hidden_state`
call (Stage1/projector_trainer.py:158-171), i.e. HF `SiglipVisionModel`
(TF/models/siglip/modeling_siglip.py:576-619) minus the MAP head whose output
the trainer discards.  Weights are HF-named (`vision_model.*`), converted once
into the kernel layout: fused q|k|v rows, conv weight flattened (c, ky, kx),
GEMM weights bf16, biases/LN/positions fp32.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib as L
from . import kernels as K
from .config import SiglipVisionConfig


def _dev(a, dtype, device):
    t = torch.from_numpy(a) if isinstance(a, np.ndarray) else a
    return t.to(device=device, dtype=dtype).contiguous()


class SiglipVisionTower:
    def __init__(self, cfg: SiglipVisionConfig, params: dict, device="cuda", prefix="vision_model."):
        self.cfg, self.device = cfg, torch.device(device)
        bf, f32 = torch.bfloat16, torch.float32
        g = lambda n, dt: _dev(params[prefix + n], dt, self.device)
        D = cfg.hidden_size
        self.patch_w = g("embeddings.patch_embedding.weight", bf).reshape(D, -1).contiguous()
        self.patch_b = g("embeddings.patch_embedding.bias", f32)
        self.pos = g("embeddings.position_embedding.weight", f32)
        self.post_w, self.post_b = g("post_layernorm.weight", f32), g("post_layernorm.bias", f32)
        self.layers = []
        for i in range(cfg.num_hidden_layers):
            p = f"encoder.layers.{i}."
            lay = dict(
                wqkv=torch.cat([g(p + f"self_attn.{n}_proj.weight", bf) for n in "qkv"]).contiguous(),
                bqkv=torch.cat([g(p + f"self_attn.{n}_proj.bias", f32) for n in "qkv"]).contiguous(),
                wo=g(p + "self_attn.out_proj.weight", bf), bo=g(p + "self_attn.out_proj.bias", f32),
                w1=g(p + "mlp.fc1.weight", bf), b1=g(p + "mlp.fc1.bias", f32),
                w2=g(p + "mlp.fc2.weight", bf), b2=g(p + "mlp.fc2.bias", f32),
                ln1_w=g(p + "layer_norm1.weight", f32), ln1_b=g(p + "layer_norm1.bias", f32),
                ln2_w=g(p + "layer_norm2.weight", f32), ln2_b=g(p + "layer_norm2.bias", f32))
            self.layers.append(lay)
        self._build_c()
        self._ws = None

    @classmethod
    def from_hf(cls, model, device="cuda"):
        """From an HF SiglipModel / SiglipVisionModel instance."""
        vm = model.vision_model if hasattr(model, "vision_model") else model
        vc = vm.config
        cfg = SiglipVisionConfig(image_size=vc.image_size, patch_size=vc.patch_size, num_channels=vc.num_channels,
                                 hidden_size=vc.hidden_size, num_attention_heads=vc.num_attention_heads,
                                 intermediate_size=vc.intermediate_size, num_hidden_layers=vc.num_hidden_layers,
                                 layer_norm_eps=vc.layer_norm_eps)
        sd = {"vision_model." + k: v.detach().float() for k, v in vm.state_dict().items()}
        return cls(cfg, sd, device)

    @classmethod
    def random_init(cls, cfg: SiglipVisionConfig, device="cuda", seed=0):
        """Synthetic weights generated on the device (benchmark: no checkpoints offline)."""
        dev = torch.device(device)
        self = cls.__new__(cls)
        self.cfg, self.device = cfg, dev
        D, I = cfg.hidden_size, cfg.intermediate_size
        s = [seed * 1000]

        def nb(*shape, std=0.02):
            s[0] += 1
            return K.fill_normal_(torch.empty(shape, dtype=torch.bfloat16, device=dev), s[0], std)
        f = lambda n, v=0.0: torch.full((n,), v, dtype=torch.float32, device=dev)
        self.patch_w = nb(D, cfg.patch_dim)
        self.patch_b = f(D)
        self.pos = nb(cfg.num_patches, D).float()
        self.post_w, self.post_b = f(D, 1.0), f(D)
        self.layers = [dict(wqkv=nb(3 * D, D), bqkv=f(3 * D), wo=nb(D, D), bo=f(D), w1=nb(I, D), b1=f(I),
                            w2=nb(D, I), b2=f(D), ln1_w=f(D, 1.0), ln1_b=f(D), ln2_w=f(D, 1.0), ln2_b=f(D))
                       for _ in range(cfg.num_hidden_layers)]
        self._build_c()
        self._ws = None
        return self

    def _build_c(self):
        c = self.cfg
        self.c_cfg = L.SiglipConfigC(c.image_size, c.patch_size, c.num_channels, c.hidden_size,
                                     c.num_attention_heads, c.intermediate_size, c.num_hidden_layers,
                                     c.layer_norm_eps)
        arr = (L.SiglipLayerC * len(self.layers))()
        for i, lay in enumerate(self.layers):
            arr[i] = L.SiglipLayerC(*[lay[k].data_ptr() for k in ("wqkv", "bqkv", "wo", "bo", "w1", "b1", "w2", "b2",
                                                                   "ln1_w", "ln1_b", "ln2_w", "ln2_b")])
        self._c_layers = arr
        self.c_w = L.SiglipWeightsC(self.patch_w.data_ptr(), self.patch_b.data_ptr(), self.pos.data_ptr(),
                                    self.post_w.data_ptr(), self.post_b.data_ptr(),
                                    C.cast(arr, C.POINTER(L.SiglipLayerC)))

    def workspace(self, batch):
        n = L.lib().ptk_siglip_workspace_bytes(self.c_cfg, batch)
        if self._ws is None or self._ws.numel() < n:
            self._ws = torch.empty(n, dtype=torch.uint8, device=self.device)
        return self._ws

    def forward_into(self, pixels_bf16, out):
        """pixels bf16 [B,C,H,W] -> out bf16 [B*N, D] (last_hidden_state, all patches)."""
        B = pixels_bf16.shape[0]
        ws = self.workspace(B)
        L.check(L.lib().ptk_siglip_fwd(self.c_cfg, self.c_w, B, pixels_bf16.data_ptr(), out.data_ptr(),
                                       ws.data_ptr(), ws.numel(), L.stream_ptr(self.device)), "ptk_siglip_fwd")
        return out

    def __call__(self, pixel_values):
        """HF-style: pixel_values [B,C,H,W] (any float dtype) -> last_hidden_state bf16 [B,N,D]."""
        if not pixel_values.is_cuda:
            raise L.PtkError("SiglipVisionTower runs on the HIP device only")
        px = pixel_values.to(torch.bfloat16).contiguous()
        B = px.shape[0]
        out = torch.empty((B * self.cfg.num_patches, self.cfg.hidden_size), dtype=torch.bfloat16, device=self.device)
        self.forward_into(px, out)
        return out.view(B, self.cfg.num_patches, self.cfg.hidden_size)
