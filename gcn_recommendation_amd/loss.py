"""BPR-loss API kept from the reference (main.py:366-402), callable exactly as main.py:515-522.

The loss itself is B=2048 rows of d-wide dot products — negligible next to the propagation — so
it is plain torch (on a HIP device its ops run as ROCm kernels). Signature, defaults and
arithmetic order match the reference: BPR = -mean(log(sigmoid(pos - neg) + 1e-8)), optional
brand BPR weighted by brand_loss_weight, L2 of the layer-0 rows / batch size.
"""
import torch


def bpr_loss_reg(final_user_emb, final_pos_item_emb, final_neg_item_emb,
                 initial_user_emb, initial_pos_item_emb, initial_neg_item_emb,
                 lambda_reg,
                 brand_loss=False,
                 final_brand_emb=None,
                 pos_item_brand_idx=None,
                 neg_item_brand_idx=None,
                 brand_loss_weight=0.1):
    pos_scores = torch.sum(final_user_emb * final_pos_item_emb, dim=1)
    neg_scores = torch.sum(final_user_emb * final_neg_item_emb, dim=1)
    bpr_loss = -torch.mean(torch.log(torch.sigmoid(pos_scores - neg_scores) + 1e-8))

    brand_loss_val = 0.0
    if brand_loss and final_brand_emb is not None:
        pos_brand_emb = final_brand_emb[pos_item_brand_idx]
        neg_brand_emb = final_brand_emb[neg_item_brand_idx]
        brand_pos_score = torch.sum(final_user_emb * pos_brand_emb, dim=1)
        brand_neg_score = torch.sum(final_user_emb * neg_brand_emb, dim=1)
        brand_loss_val = -torch.mean(torch.log(torch.sigmoid(brand_pos_score - brand_neg_score)
                                               + 1e-8))

    reg_loss = lambda_reg * (
        initial_user_emb.norm(2).pow(2)
        + initial_pos_item_emb.norm(2).pow(2)
        + initial_neg_item_emb.norm(2).pow(2)
    ) / float(len(final_user_emb))
    return bpr_loss + brand_loss_weight * brand_loss_val + reg_loss
