"""BPR-loss API kept from the reference (main.py:366-402), callable exactly as main.py:515-522.

On a HIP device the base BPR term and the L2 term run as ONE fused kernel (lgcn_bpr_loss,
csrc/lgcn_bpr.hip): both dot products, log-sigmoid, the squared norms of the layer-0 rows and
all six input gradients in one pass, the batch mean in a fixed order. On CPU tensors the
reference's own torch expression runs (device dispatch, as the models do). The brand-loss branch
(dead in the reference snapshot: main.py:505/509 never define item_to_brand) stays the
reference's torch expression on either device. Arithmetic: BPR = -mean(log(sigmoid(pos - neg)
+ 1e-8)), L2 of the layer-0 rows / batch size; fp32 reductions, so GPU parity with the
reference is a tolerance (tests/test_gpu_parity.py::test_fused_bpr_loss_vs_torch).
"""
import torch

from . import engine


class BPRLossFunction(torch.autograd.Function):
    """Fused forward; the gradients are produced by the same launch and scaled on backward."""

    @staticmethod
    def forward(ctx, u, p, n, u0, p0, n0, lambda_reg):
        lib = engine.load_library()
        B, d = u.shape
        xs = [t.detach() for t in (u, p, n, u0, p0, n0)]
        for t in xs:
            if t.shape != (B, d) or t.dtype != torch.float32 or t.stride(1) != 1:
                raise engine.LgcnError("bpr_loss: six [B x d] fp32 row-major blocks expected")
        dev = u.device
        terms = torch.empty(2 * B, dtype=torch.float32, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        grads = torch.empty((6, B, d), dtype=torch.float32, device=dev)
        args = []
        for t in xs:
            args += [engine._ptr(t), t.stride(0)]
        with torch.cuda.device(dev):
            engine._check(lib.lgcn_bpr_loss(*args, B, d, float(lambda_reg), engine._ptr(terms),
                                            engine._ptr(loss), engine._ptr(grads),
                                            engine._stream(dev)), "lgcn_bpr_loss")
        ctx.save_for_backward(grads)
        return loss

    @staticmethod
    def backward(ctx, g):
        (grads,) = ctx.saved_tensors
        return tuple(grads[i] * g for i in range(6)) + (None,)


def _torch_bpr(u, p, n):
    pos_scores = torch.sum(u * p, dim=1)
    neg_scores = torch.sum(u * n, dim=1)
    return -torch.mean(torch.log(torch.sigmoid(pos_scores - neg_scores) + 1e-8))


def bpr_loss_reg(final_user_emb, final_pos_item_emb, final_neg_item_emb,
                 initial_user_emb, initial_pos_item_emb, initial_neg_item_emb,
                 lambda_reg,
                 brand_loss=False,
                 final_brand_emb=None,
                 pos_item_brand_idx=None,
                 neg_item_brand_idx=None,
                 brand_loss_weight=0.1):
    brand_loss_val = 0.0
    if brand_loss and final_brand_emb is not None:
        pos_brand_emb = final_brand_emb[pos_item_brand_idx]
        neg_brand_emb = final_brand_emb[neg_item_brand_idx]
        brand_loss_val = _torch_bpr(final_user_emb, pos_brand_emb, neg_brand_emb)

    if final_user_emb.device.type == "cuda":
        base = BPRLossFunction.apply(final_user_emb, final_pos_item_emb, final_neg_item_emb,
                                     initial_user_emb, initial_pos_item_emb,
                                     initial_neg_item_emb, float(lambda_reg))
        return base + brand_loss_weight * brand_loss_val if brand_loss_val != 0.0 else base

    bpr_loss = _torch_bpr(final_user_emb, final_pos_item_emb, final_neg_item_emb)
    reg_loss = lambda_reg * (
        initial_user_emb.norm(2).pow(2)
        + initial_pos_item_emb.norm(2).pow(2)
        + initial_neg_item_emb.norm(2).pow(2)
    ) / float(len(final_user_emb))
    return bpr_loss + brand_loss_weight * brand_loss_val + reg_loss
