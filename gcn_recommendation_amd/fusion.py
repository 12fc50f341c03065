"""The LightGCN_Fusion item pre-layer (reference models/lightgcn_fusion.py:45-49)

    fused_item_emb_0 = F.leaky_relu(item_fusion_layer(torch.cat([item_id_emb_0, content], 1)))

on a HIP device as one kernel (lgcn_fusion_prelayer: no concatenation, exact-f32 MFMA GEMM,
bias + leaky_relu in its epilogue). The backward is the same arithmetic autograd would run for
the reference expression, written out with torch ops (training only): g = dF where F > 0, else
slope * dF; d_id = g · W[:, :d]; dW = gᵀ · [id | content]; db = Σ g. The content table is a
buffer (no gradient), as in the reference.
"""

import torch

from . import engine

SUPPORTED_D = (64, 128)
SUPPORTED_C = (32, 64, 128)


def supported(d, c_dim):
    return d in SUPPORTED_D and c_dim in SUPPORTED_C


class FusionPreLayer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, id_w, content, weight, bias, slope):
        lib = engine.load_library()
        n, d = id_w.shape
        c_dim = content.shape[1]
        idc, cc = id_w.detach().contiguous(), content.detach().contiguous()
        wc = weight.detach().contiguous()
        bc = bias.detach().contiguous() if bias is not None else None
        out = torch.empty((n, d), dtype=torch.float32, device=id_w.device)
        with torch.cuda.device(id_w.device):
            engine._check(lib.lgcn_fusion_prelayer(
                engine._ptr(idc), idc.stride(0) if n else d, engine._ptr(cc),
                cc.stride(0) if n else c_dim, n, d, c_dim, engine._ptr(wc), engine._ptr(bc),
                float(slope), engine._ptr(out), d, engine._stream(id_w.device)),
                "lgcn_fusion_prelayer")
        ctx.save_for_backward(idc, cc, wc, out)
        ctx.slope = slope
        ctx.has_bias = bias is not None
        return out

    @staticmethod
    def backward(ctx, g_out):
        idc, cc, wc, out = ctx.saved_tensors
        d = idc.shape[1]
        g = torch.where(out > 0, g_out, g_out * ctx.slope)
        d_id = g @ wc[:, :d] if ctx.needs_input_grad[0] else None
        d_w = None
        if ctx.needs_input_grad[2]:
            d_w = torch.cat([g.t() @ idc, g.t() @ cc], 1)
        d_b = g.sum(0) if ctx.has_bias and ctx.needs_input_grad[3] else None
        return d_id, None, d_w, d_b, None


def fused_item_embedding(id_w, content, linear, slope=0.01):
    """leaky_relu(linear(cat([id_w, content], 1))) — the engine kernel on a HIP device for the
    supported shapes, the reference's torch ops otherwise (CPU tensors, other dims)."""
    if id_w.device.type == "cuda" and supported(id_w.shape[1], content.shape[1]) and \
            linear.weight.shape == (id_w.shape[1], id_w.shape[1] + content.shape[1]):
        return FusionPreLayer.apply(id_w, content, linear.weight, linear.bias, slope)
    combined = torch.cat([id_w, content], dim=1)
    return torch.nn.functional.leaky_relu(linear(combined), slope)
