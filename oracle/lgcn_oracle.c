/*
 * lgcn_oracle.c — TEST INFRASTRUCTURE ONLY. CPU restatement of the reference's propagation
 * arithmetic, used as the parity checker. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product (gcn_recommendation_amd/, models/) never does.
 *
 * Pinned against the reference: tests/test_oracle_golden.py checks every function below
 * bitwise against the golden vectors that tests/golden/gen_golden.py produced by importing the
 * reference (sha1 of every layer, the final embeddings and the embedding gradients).
 *
 * What it restates:
 *  - torch.sparse.mm(adj_mat, ego) as called at models/lightgcn.py:45: on CPU, ATen's
 *    addmm_sparse_dense worker zeroes the result, then for every stored nonzero j in stored order
 *    does r[row_j,:] = fma(val_j, dense[col_j,:], r[row_j,:]) (a cpublas axpy; MKL's saxpy uses
 *    FMA). Third-party arithmetic: PyTorch (unpinned by the reference; torch 2.10.0 here).
 *  - torch.mean(torch.stack([E0..EK]), 0) (models/lightgcn.py:54): ((E0+E1)+...+EK)/(K+1),
 *    sequential, correctly rounded division (holds for K+1 <= 17; checked in tests).
 *  - The autograd backward of lines 40-54 for an upstream gradient G: MeanBackward gives every
 *    layer G/(K+1); SparseAddmmBackward0 gives Âᵀ·dE_{k+1}; accumulation is
 *    dE_k = G/(K+1) + Âᵀ·dE_{k+1} (addition commutes bitwise), i.e. the Horner recurrence.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off; fmaf is the only fused operation).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* Y[n_rows x d] = Â·X for a COO given in stored order (rows/cols int64, vals fp32). */
void oracle_spmm_coo(int64_t nnz, const int64_t* rows, const int64_t* cols, const float* vals,
                     int64_t n_rows, int64_t d, const float* x, float* y) {
    memset(y, 0, sizeof(float) * (size_t)(n_rows * d));
    for (int64_t j = 0; j < nnz; ++j) {
        const float v = vals[j];
        const float* xr = x + cols[j] * d;
        float* yr = y + rows[j] * d;
        for (int64_t c = 0; c < d; ++c) yr[c] = fmaf(v, xr[c], yr[c]);
    }
}

/* Selected rows of Â·X: y[i,:] = row sel[i] of oracle_spmm_coo's result. A row's value is the
 * chain over its own nonzeros only, in stored order, so for a row-sorted COO (main.py:331-336
 * stores one) the chain of row r is nonzeros rowptr[r]..rowptr[r+1]-1 — the same fmaf sequence
 * oracle_spmm_coo runs for it. Rows are independent: OpenMP over the selection. Used by the
 * full-size GPU parity tests (BASELINE configs at 56M nonzeros), which check sampled rows of
 * every layer against this with the GPU's previous layer as X. */
void oracle_spmm_rows(const int64_t* rowptr, const int64_t* cols, const float* vals, int64_t d,
                      const float* x, int64_t n_sel, const int64_t* sel, float* y) {
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t i = 0; i < n_sel; ++i) {
        float* yr = y + i * d;
        for (int64_t c = 0; c < d; ++c) yr[c] = 0.0f;
        for (int64_t j = rowptr[sel[i]]; j < rowptr[sel[i] + 1]; ++j) {
            const float v = vals[j];
            const float* xr = x + cols[j] * d;
            for (int64_t c = 0; c < d; ++c) yr[c] = fmaf(v, xr[c], yr[c]);
        }
    }
}

/* lightgcn.py:40-54 — final[n x d] = mean(E0..EK). layers_out (optional) receives E1..EK
 * back to back ([K][n][d]). */
void oracle_forward(int64_t nnz, const int64_t* rows, const int64_t* cols, const float* vals,
                    int64_t n, int64_t d, int64_t K, const float* e0, float* final_out,
                    float* layers_out) {
    const size_t sz = (size_t)(n * d);
    float* prev = (float*)malloc(sizeof(float) * (sz ? sz : 1));
    float* cur = (float*)malloc(sizeof(float) * (sz ? sz : 1));
    memcpy(final_out, e0, sizeof(float) * sz);  /* running sum starts at E0 */
    memcpy(prev, e0, sizeof(float) * sz);
    for (int64_t k = 0; k < K; ++k) {
        oracle_spmm_coo(nnz, rows, cols, vals, n, d, prev, cur);
        for (size_t i = 0; i < sz; ++i) final_out[i] = final_out[i] + cur[i];
        if (layers_out) memcpy(layers_out + (size_t)k * sz, cur, sizeof(float) * sz);
        float* t = prev; prev = cur; cur = t;
    }
    const float div = (float)(K + 1);
    for (size_t i = 0; i < sz; ++i) final_out[i] = final_out[i] / div;
    free(prev);
    free(cur);
}

/* Backward of lightgcn.py:40-54 for upstream G: grad_e0 = dE0. `rows/cols` are Â's COO (the
 * transpose is taken here, keeping stored order, as torch's sparse t() does). */
void oracle_backward(int64_t nnz, const int64_t* rows, const int64_t* cols, const float* vals,
                     int64_t n, int64_t d, int64_t K, const float* g, float* grad_e0) {
    const size_t sz = (size_t)(n * d);
    float* c = (float*)malloc(sizeof(float) * (sz ? sz : 1));
    float* h = (float*)malloc(sizeof(float) * (sz ? sz : 1));
    float* t = (float*)malloc(sizeof(float) * (sz ? sz : 1));
    const float div = (float)(K + 1);
    for (size_t i = 0; i < sz; ++i) c[i] = g[i] / div;
    memcpy(h, c, sizeof(float) * sz);
    for (int64_t k = 0; k < K; ++k) {
        oracle_spmm_coo(nnz, cols, rows, vals, n, d, h, t);  /* Âᵀ·h */
        for (size_t i = 0; i < sz; ++i) h[i] = c[i] + t[i];
    }
    memcpy(grad_e0, h, sizeof(float) * sz);
    free(c);
    free(h);
    free(t);
}

/* fp64 arbiter (not a restatement): the same propagation in double precision over a row-sorted
 * COO, OpenMP over rows. Used to measure how far the fp32 reference AND the engine are from
 * exact arithmetic on graphs whose hub rows make the reference's own rounding error exceed the
 * 1e-5 normwise gate (bench.py parity fields, tests/test_gpu_parity.py). */
void oracle_forward_f64(int64_t nnz, const int64_t* rows, const int64_t* cols, const float* vals,
                        int64_t n, int64_t d, int64_t K, const float* e0, double* final_out) {
    const size_t sz = (size_t)(n * d);
    int64_t* rowptr = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
    for (int64_t j = 0; j < nnz; ++j) rowptr[rows[j] + 1]++;
    for (int64_t r = 0; r < n; ++r) rowptr[r + 1] += rowptr[r];
    double* prev = (double*)malloc(sizeof(double) * (sz ? sz : 1));
    double* cur = (double*)malloc(sizeof(double) * (sz ? sz : 1));
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)sz; ++i) { prev[i] = e0[i]; final_out[i] = e0[i]; }
    for (int64_t k = 0; k < K; ++k) {
#pragma omp parallel for schedule(dynamic, 1024)
        for (int64_t r = 0; r < n; ++r) {
            double* yr = cur + r * d;
            for (int64_t c = 0; c < d; ++c) yr[c] = 0.0;
            for (int64_t j = rowptr[r]; j < rowptr[r + 1]; ++j) {
                const double v = vals[j];
                const double* xr = prev + cols[j] * d;
                for (int64_t c = 0; c < d; ++c) yr[c] += v * xr[c];
            }
            for (int64_t c = 0; c < d; ++c) final_out[r * d + c] += yr[c];
        }
        double* t = prev; prev = cur; cur = t;
    }
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)sz; ++i) final_out[i] /= (double)(K + 1);
    free(rowptr);
    free(prev);
    free(cur);
}
