"""MLPProjector — same API and state-dict layout as the reference
(`Stage1/projectors.py:4-29`): `.model = nn.Sequential(Linear(Dv, 10*Dv),
GELU(), Linear(10*Dv, Dl))`, keys `model.0.{weight,bias}`, `model.2.{weight,bias}`.

MI355X layout: the four fp32 master tensors are views into ONE flat buffer
(`flat`, 22.29 M fp32 for L-384 -> Gemma3-1B) and their grads into `flat_grad`,
so the gradient all-reduce is a single RCCL call and clip + AdamW is a single
fused kernel.  bf16 GEMM shadows (W1, W2, W2^T) are refreshed after each
update.  forward() runs the libptk kernels (ptk_projector_fwd/bwd) through a
torch.autograd.Function; there is no CPU path.
"""
from __future__ import annotations


import torch
import torch.nn as nn

from . import _lib as L
from . import kernels as K


class MLPProjector(nn.Module):
    def __init__(self, vision_dim: int, llm_dim: int, expansion_factor: int = 10, device=None):
        super().__init__()
        intermediate_dim = vision_dim * expansion_factor
        self.vision_dim, self.inter_dim, self.llm_dim = vision_dim, intermediate_dim, llm_dim
        self.model = nn.Sequential(nn.Linear(vision_dim, intermediate_dim), nn.GELU(),
                                   nn.Linear(intermediate_dim, llm_dim))
        if device is not None:
            self.model.to(device)
        self._flatten()

    # ------------------------------------------------------------------ storage
    def _flatten(self):
        """Re-home the 4 parameters as views of one contiguous fp32 buffer."""
        params = [self.model[0].weight, self.model[0].bias, self.model[2].weight, self.model[2].bias]
        dev = params[0].device
        n = sum(p.numel() for p in params)
        flat = torch.empty(n, dtype=torch.float32, device=dev)
        grad = torch.zeros(n, dtype=torch.float32, device=dev)
        self._views, o = [], 0
        for p in params:
            k = p.numel()
            flat[o:o + k].copy_(p.detach().reshape(-1))
            p.data = flat[o:o + k].view(p.shape)
            p.grad = grad[o:o + k].view(p.shape)
            self._views.append((o, k, tuple(p.shape)))
            o += k
        self.flat, self.flat_grad = flat, grad
        # every device-resident cache is dropped: the bf16 shadows, W1^T, the stream-K tail scratch and the
        # autograd backward's workspace / grad scratch are (re)allocated on the new device when next used
        self._w1b = None
        self._w1t = None
        self._tail = None
        self._bwd_ws = None
        self._grad_tmp = None
        self._shadow_dirty = True

    def _apply(self, fn, *args, **kw):      # keep the flat layout across .to()/.cuda()
        super()._apply(fn, *args, **kw)
        if hasattr(self, "flat") and self.model[0].weight.device != self.flat.device:
            self._flatten()
        return self

    def load_state_dict(self, state_dict, strict=True, assign=False):
        r = super().load_state_dict(state_dict, strict=strict, assign=False)
        self._shadow_dirty = True
        return r

    @property
    def w1(self):
        return self.model[0].weight

    @property
    def b1(self):
        return self.model[0].bias

    @property
    def w2(self):
        return self.model[2].weight

    @property
    def b2(self):
        return self.model[2].bias

    def grads(self):
        return [self.flat_grad[o:o + k].view(s) for o, k, s in self._views]

    def refresh_shadows(self):
        """bf16 GEMM operands from the fp32 masters (the reference's autocast cast)."""
        if not self.flat.is_cuda:
            raise L.PtkError("MLPProjector kernels need the HIP device")
        if getattr(self, "_w1b", None) is None:
            self._w1b = torch.empty(self.w1.shape, dtype=torch.bfloat16, device=self.flat.device)
            self._w2b = torch.empty(self.w2.shape, dtype=torch.bfloat16, device=self.flat.device)
            self._w2t = torch.empty((self.inter_dim, self.llm_dim), dtype=torch.bfloat16, device=self.flat.device)
            # stream-K tail scratch of the projector's GEMMs (ptk_projector.tail_ws; the fc2 projection's 104-tile
            # tail round runs split)
            self._tail = torch.zeros(L.lib().ptk_gemm_tail_scratch_bytes(), dtype=torch.uint8, device=self.flat.device)
        K.cast_bf16(self.w1.detach(), self._w1b)
        K.cast_bf16(self.w2.detach(), self._w2b)
        K.transpose(self._w2b, out=self._w2t)     # in place: no allocation per optimizer step
        if getattr(self, "_w1t", None) is not None:   # W1^T of the autograd input grad, once built
            K.transpose(self._w1b, out=self._w1t)
        self.c = L.ProjectorC(self.vision_dim, self.inter_dim, self.llm_dim, self._w1b.data_ptr(),
                              self.b1.data_ptr(), self._w2b.data_ptr(), self.b2.data_ptr(), self._w2t.data_ptr(),
                              self._tail.data_ptr() if self._tail is not None else None)
        self._shadow_dirty = False

    def desc(self):
        if self._shadow_dirty:
            self.refresh_shadows()
        return self.c

    # ------------------------------------------------------------------ kernels
    def fwd_into(self, x_bf16, a, h, out, out_map=(0, 0, 0, 0), ld_out=None, round_bf16=True):
        rows = x_bf16.shape[0]
        L.check(L.lib().ptk_projector_fwd(self.desc(), rows, x_bf16.data_ptr(), a.data_ptr(), h.data_ptr(),
                                          out.data_ptr(), L.RowMap(*out_map),
                                          self.llm_dim if ld_out is None else ld_out, int(round_bf16),
                                          L.stream_ptr(x_bf16.device)), "ptk_projector_fwd")

    def workspace_bytes(self, rows):
        return L.lib().ptk_projector_workspace_bytes(self.desc(), rows)

    def bwd_into(self, x_bf16, a, h, dy_bf16, ws):
        """Writes the 4 parameter grads into flat_grad (overwrite)."""
        rows = x_bf16.shape[0]
        g = self.grads()
        L.check(L.lib().ptk_projector_bwd(self.desc(), rows, x_bf16.data_ptr(), a.data_ptr(), h.data_ptr(),
                                          dy_bf16.data_ptr(), g[0].data_ptr(), g[1].data_ptr(), g[2].data_ptr(),
                                          g[3].data_ptr(), ws.data_ptr(), ws.numel(), L.stream_ptr(x_bf16.device)),
                "ptk_projector_bwd")

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x [B, N, Dv] -> [B, N, Dl] (fp32 output of bf16 GEMMs, as under autocast)."""
        if not x.is_cuda:
            raise L.PtkError("MLPProjector.forward runs on the HIP device only")
        return _ProjectorFn.apply(x, self.flat, self)


class _ProjectorFn(torch.autograd.Function):
    """Autograd of `self.model(x)` under the reference's bf16 autocast (Stage1/projectors.py:22-29):
    the parameter grads accumulate into flat_grad (as `.grad` does), and the input grad is
    dX = ((dY . W2) * gelu'(a)) . W1 -- the chain the reference's autograd takes through fc2, GELU and fc1,
    with bf16 GEMM operands and the bf16 intermediate dA that autocast produces."""

    @staticmethod
    def forward(ctx, x, flat, mod: MLPProjector):
        shp = x.shape
        xb = x.reshape(-1, shp[-1]).to(torch.bfloat16).contiguous()
        R = xb.shape[0]
        a = torch.empty((R, mod.inter_dim), dtype=torch.bfloat16, device=x.device)
        h = torch.empty_like(a)
        out = torch.empty((R, mod.llm_dim), dtype=torch.float32, device=x.device)
        mod.fwd_into(xb, a, h, out)
        ctx.save_for_backward(xb, a, h)
        ctx.mod, ctx.x_shape, ctx.x_dtype = mod, shp, x.dtype
        return out.view(*shp[:-1], mod.llm_dim)

    @staticmethod
    def backward(ctx, gout):
        xb, a, h = ctx.saved_tensors
        mod = ctx.mod
        dy = gout.reshape(-1, mod.llm_dim).to(torch.bfloat16).contiguous()
        # workspace and grad scratch kept on the module across calls (grown when a larger batch comes)
        nb = mod.workspace_bytes(xb.shape[0])
        if getattr(mod, "_bwd_ws", None) is None or mod._bwd_ws.numel() < nb:
            mod._bwd_ws = torch.empty(nb, dtype=torch.uint8, device=xb.device)
        if getattr(mod, "_grad_tmp", None) is None:
            mod._grad_tmp = torch.empty_like(mod.flat_grad)
        g = [mod._grad_tmp[o:o + k] for o, k, _ in mod._views]
        L.check(L.lib().ptk_projector_bwd(mod.desc(), xb.shape[0], xb.data_ptr(), a.data_ptr(), h.data_ptr(),
                                          dy.data_ptr(), g[0].data_ptr(), g[1].data_ptr(), g[2].data_ptr(),
                                          g[3].data_ptr(), mod._bwd_ws.data_ptr(), mod._bwd_ws.numel(),
                                          L.stream_ptr(xb.device)), "ptk_projector_bwd")
        mod.flat_grad.add_(mod._grad_tmp)   # accumulate like autograd would
        dx = None
        if ctx.needs_input_grad[0]:
            # dA = (dY . W2) * gelu'(a) (bf16, the fused GELU-backward epilogue), then dX = dA . W1
            da = K.gemm(dy, mod._w2t, act=L.ACT_GELU_ERF_BWD, aux_in=a)
            if getattr(mod, "_w1t", None) is None:   # [Dv, I]: W1 as the K-contiguous B operand (cached)
                mod._w1t = K.transpose(mod._w1b)
            dx = K.gemm(da, mod._w1t, out_dtype=torch.float32)
            dx = dx.view(*ctx.x_shape).to(ctx.x_dtype)
        return dx, None, None
