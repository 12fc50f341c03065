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
