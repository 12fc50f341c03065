"""Recall@K / NDCG@K on device (the semantics of main.py:404-439).

Scores = user rows · item tableᵀ (hipBLASLt via torch.matmul), every training item of the user
masked to -1e10 (main.py:422-424), topk(K) (main.py:426), hit -> recall 1, NDCG 1/log2(pos+2)
(main.py:430-438). The training items come straight from the engine's CSR (a user's row holds its
items at column offset U), so no Python loop over users is needed.
"""
import numpy as np
import torch


def recall_ndcg(user_emb, item_emb, users, heldout_items, train_rowptr, train_cols, U, k=20,
                batch_size=1024, return_topk=False):
    """users: int64 [n] user ids; heldout_items: int64 [n] item ids (one per user);
    train_rowptr/train_cols: host CSR of Â (numpy) — a user row's cols >= U are its items."""
    dev = user_emb.device
    users = np.asarray(users, dtype=np.int64)
    heldout_items = np.asarray(heldout_items, dtype=np.int64)
    hits, ndcgs, tops = [], [], []
    with torch.no_grad():
        for s in range(0, len(users), batch_size):
            bu = users[s:s + batch_size]
            scores = torch.matmul(user_emb[torch.from_numpy(bu).to(dev)], item_emb.T)
            lens = train_rowptr[bu + 1] - train_rowptr[bu]
            rr = np.repeat(np.arange(len(bu)), lens)
            cc = np.concatenate([train_cols[train_rowptr[u]:train_rowptr[u + 1]] for u in bu]) \
                if lens.sum() else np.zeros(0, np.int64)
            keep = cc >= U
            if keep.any():
                scores[torch.from_numpy(rr[keep]).to(dev),
                       torch.from_numpy(cc[keep] - U).to(dev)] = -1e10
            _, top = torch.topk(scores, k=k)
            top = top.cpu().numpy()
            if return_topk:
                tops.append(top)
            truth = heldout_items[s:s + batch_size]
            for j in range(len(bu)):
                pos = np.nonzero(top[j] == truth[j])[0]
                hits.append(1 if pos.size else 0)
                ndcgs.append(1 / np.log2(pos[0] + 2) if pos.size else 0)
    if return_topk:
        return float(np.mean(hits)), float(np.mean(ndcgs)), np.concatenate(tops)
    return float(np.mean(hits)), float(np.mean(ndcgs))


# ----------------------------------------------------------------------------------------------
# fused path: lgcn_score_topk (score GEMM + train mask + top-K in one kernel, no score matrix)
# ----------------------------------------------------------------------------------------------
def mask_csr(users, items, n_users):
    """Sorted, de-duplicated per-user item lists (the train_user_items dict of main.py:407)."""
    users = np.asarray(users, dtype=np.int64)
    items = np.asarray(items, dtype=np.int64)
    key = np.unique(users * (items.max(initial=0) + 1) + items) if users.size else users
    if users.size:
        span = items.max(initial=0) + 1
        u, it = key // span, key % span
    else:
        u, it = users, items
    rowptr = np.searchsorted(u, np.arange(n_users + 1)).astype(np.int32)
    return rowptr, it.astype(np.int32)


def topk_fused(user_emb, item_emb, users, mask_rowptr, mask_items, k=20):
    """Top-k items per user (scores, indices) with the train items masked to -1e10.
    user_emb [U x d], item_emb [I x d] fp32 on the HIP device; users: int32/int64 ids."""
    import ctypes
    from . import engine
    lib = engine.load_library()
    dev = item_emb.device
    d = item_emb.shape[1]
    users = torch.as_tensor(users, device=dev).to(torch.int32).contiguous()
    n = int(users.numel())
    ue, ie = user_emb.contiguous(), item_emb.contiguous()
    mrow = torch.as_tensor(mask_rowptr, device=dev).to(torch.int32).contiguous()
    mit = torch.as_tensor(mask_items, device=dev).to(torch.int32).contiguous()
    if mit.numel() == 0:
        mit = torch.zeros(1, dtype=torch.int32, device=dev)
    n_cu = ctypes.c_int32(0)
    engine._check(lib.lgcn_device_info(dev.index or 0, ctypes.byref(n_cu), None), "device_info")
    splits = lib.lgcn_eval_splits(n, int(ie.shape[0]), n_cu.value)
    part_s = torch.empty((splits, max(n, 1), k), dtype=torch.float32, device=dev)
    part_i = torch.empty((splits, max(n, 1), k), dtype=torch.int32, device=dev)
    top_s = torch.empty((max(n, 1), k), dtype=torch.float32, device=dev)
    top_i = torch.empty((max(n, 1), k), dtype=torch.int32, device=dev)
    P = engine._ptr
    with torch.cuda.device(dev):
        engine._check(lib.lgcn_score_topk(P(ue), ue.stride(0), P(users), n, P(ie), ie.stride(0),
                                          int(ie.shape[0]), d, P(mrow), P(mit), k, splits,
                                          P(part_s), P(part_i), P(top_s), P(top_i),
                                          engine._stream(dev)), "lgcn_score_topk")
    return top_s[:n], top_i[:n]


FUSED_DIMS = (32, 64, 128, 256)   # lgcn_score_topk's widths (include/lgcn.h)
FUSED_MAX_K = 32


def fused_supported(d, k):
    return d in FUSED_DIMS and 1 <= k <= FUSED_MAX_K


def topk_torch(user_emb, item_emb, users, mask_rowptr, mask_items, k=20):
    """main.py:420-426 as torch ops for any d and k: scores = user rows · item tableᵀ, every
    training item of the user set to -1e10, topk(k)."""
    dev = item_emb.device
    users = np.asarray(users, dtype=np.int64)
    scores = torch.matmul(user_emb[torch.from_numpy(users).to(dev)], item_emb.T)
    lens = mask_rowptr[users + 1] - mask_rowptr[users]
    if lens.sum():
        rr = np.repeat(np.arange(len(users)), lens)
        cc = np.concatenate([mask_items[mask_rowptr[u]:mask_rowptr[u + 1]] for u in users])
        scores[torch.from_numpy(rr).to(dev), torch.from_numpy(cc.astype(np.int64)).to(dev)] = -1e10
    return torch.topk(scores, k=k)


def evaluate(model, val_or_test_data, train_data, norm_adj_tensor, k, device, batch_size=8192,
             use_brand=True, item_brand_df=None):
    """main.py:404-439 (same signature and metrics): one propagation, then per batch of users
    one lgcn_score_topk launch (fused score + mask + top-k) when the width and k are ones the
    kernel has (d in FUSED_DIMS, k <= FUSED_MAX_K), torch matmul + mask + topk otherwise — the
    reference works for any d and k, so does this; hit -> recall 1, NDCG = 1/log2(pos + 2)."""
    model.eval()
    test_user_items = dict(zip(val_or_test_data["user_idx"], val_or_test_data["item_idx"]))
    test_users = np.fromiter(test_user_items.keys(), dtype=np.int64, count=len(test_user_items))
    truth = np.fromiter(test_user_items.values(), dtype=np.int64, count=len(test_user_items))
    with torch.no_grad():
        all_user_emb, all_item_emb, _, _, _ = model(norm_adj_tensor)
        mrow, mit = mask_csr(train_data["user_idx"].to_numpy(), train_data["item_idx"].to_numpy(),
                             all_user_emb.shape[0])
        fused = fused_supported(all_item_emb.shape[1], k) and all_item_emb.is_cuda
        tops = []
        for s in range(0, len(test_users), batch_size):
            bu = test_users[s:s + batch_size]
            if fused:
                _, ti = topk_fused(all_user_emb, all_item_emb, bu, mrow, mit, k)
            else:
                _, ti = topk_torch(all_user_emb, all_item_emb, bu, mrow, mit, k)
            tops.append(ti.cpu().numpy())
    top = np.concatenate(tops) if tops else np.zeros((0, k), np.int32)
    hit = top == truth[:, None]
    found = hit.any(1)
    pos = hit.argmax(1)
    ndcg = np.where(found, 1.0 / np.log2(pos + 2), 0.0)
    return float(found.mean()) if len(found) else float("nan"), \
        float(ndcg.mean()) if len(found) else float("nan")
