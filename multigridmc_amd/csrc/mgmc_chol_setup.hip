// mgmc_chol_setup.hip -- the coarsest level's Cholesky factors (CholeskySampler, cholesky_sampler.cc:9-38: the banded
// precision, its factor, the dense inverses or the blocked banded solve's blocks) for the coarse Cholesky
// sampler and the exact solver's coarse solve.
#include "mgmc_internal.hpp"

namespace mgmc_host {

// banded precision of the coarsest level (+ B Sigma^{-1} B^T: cholesky_sampler.cc:30-36, the oracle's
// order), its Cholesky factor (mgmc_cholesky.hpp, bitwise the dense loop) and either the dense
// inverses G, L^{-1} (n <= CHOL_MAX_N, O(n^3) on the host) or the blocked banded solve's blocks
// (above, or MGMC_DISABLE=chol_dense; O(n bw^2)).  The bandwidth is the widest nonzero coupling:
// matrix / stencil entries and the row span of each low-rank column (the oracle computes the same).
int build_coarse_chol(mgmc_handle* h, const std::vector<LRColumn>* cols, const double* sigma, int m) {
    if (h->debug_fail_chol > 0) {  // (testing hook, mgmc_debug_fail_coarse_factor)
        --h->debug_fail_chol;
        return fail(h, MGMC_E_NOMEM, "coarse Cholesky factor: injected failure (mgmc_debug_fail_coarse_factor)");
    }
    const Level& lv = h->levels.back();
    const long long n = (long long)lv.spec.ndof;
    const bool blocked = n > CHOL_MAX_N || (h->paths & PATH_NO_CHOL_DENSE);
    const int dim = lv.spec.dim;
    const int nx = lv.spec.n[0], ny = lv.spec.n[1], nz = dim == 3 ? lv.spec.n[2] : 2;
    // the couplings (row, column, value) of the level's matrix, in the dense assembly's order
    auto for_each_entry = [&](auto&& fn) {
        if (h->field_mode) {  // the coarsest Galerkin matrix itself
            const CsrHost& A = h->coarse_csr;
            for (long long r = 0; r < n; ++r)
                for (int64_t q = A.rowptr[r]; q < A.rowptr[r + 1]; ++q) fn(r, (long long)A.col[q], A.val[q]);
            return;
        }
        for (long long r = 0; r < n; ++r) {
            const int i = (int)(r % (nx - 1)) + 1, j = (int)((r / (nx - 1)) % (ny - 1)) + 1;
            const int k = dim == 3 ? (int)(r / ((long long)(nx - 1) * (ny - 1))) + 1 : 1;
            for (int dz = (dim == 3 ? -1 : 0); dz <= (dim == 3 ? 1 : 0); ++dz)
                for (int dy = -1; dy <= 1; ++dy)
                    for (int dx = -1; dx <= 1; ++dx) {
                        const int ii = i + dx, jj = j + dy, kk = k + dz;
                        if (ii < 1 || ii > nx - 1 || jj < 1 || jj > ny - 1 || (dim == 3 && (kk < 1 || kk > nz - 1)))
                            continue;
                        const double v = dim == 3 ? lv.spec.st[(dz + 1) * 9 + (dy + 1) * 3 + (dx + 1)]
                                                  : lv.spec.st[(dy + 1) * 3 + (dx + 1)];
                        fn(r, ((long long)(dim == 3 ? kk - 1 : 0) * (ny - 1) + (jj - 1)) * (nx - 1) + (ii - 1), v);
                    }
        }
    };
    long long bw = 0;
    for_each_entry([&](long long r, long long c, double v) {
        if (v != 0.0) bw = std::max(bw, r > c ? r - c : c - r);
    });
    for (int k = 0; k < m; ++k) {
        long long lo = n, hi = -1;
        for (const auto& e : (*cols)[k].ent)
            if (e.second != 0.0) {
                lo = std::min(lo, (long long)e.first);
                hi = std::max(hi, (long long)e.first);
            }
        if (hi > lo) bw = std::max(bw, hi - lo);
    }
    const long long B = chol_block_size(bw);
    if (blocked && B > CHOL_BLOCK_MAX)
        return fail(h, MGMC_E_UNSUPPORTED,
                    "coarse Cholesky: " + std::to_string(n) + " unknowns (above " + std::to_string(CHOL_MAX_N) +
                        ") need a bandwidth of at most " + std::to_string(CHOL_BLOCK_MAX) + ", this level has " +
                        std::to_string(bw));
    if (!blocked && n > CHOL_MAX_N)
        return fail(h, MGMC_E_UNSUPPORTED, "coarse Cholesky: too many unknowns");
    // the banded host factor costs n bw^2 / 2 multiply-adds: refuse what would take more than a few
    // minutes on one core (3D 128^3 nlevel 2: 63^3 unknowns, bandwidth 4033 -- a fill-reducing sparse
    // factorisation, the reference's CHOLMOD, is the tool for such levels)
    if (blocked && (double)n * (double)bw * (double)bw > CHOL_HOST_WORK_MAX)
        return fail(h, MGMC_E_UNSUPPORTED,
                    "coarse Cholesky: " + std::to_string(n) + " unknowns of bandwidth " + std::to_string(bw) +
                        " exceed the banded factor's host work limit (n bw^2 <= " +
                        std::to_string((long long)CHOL_HOST_WORK_MAX) + "); use more levels");
    const long long W = bw + 1;
    std::vector<double> band((size_t)(n * W), 0.0);
    for_each_entry([&](long long r, long long c, double v) {
        if (c <= r && r - c <= bw) band[(size_t)(r * W + (c - r + bw))] = v;
    });
    if (m > 0) {
        std::vector<double> Bd((size_t)n * m, 0.0);
        for (int k = 0; k < m; ++k)
            for (const auto& e : (*cols)[k].ent) Bd[(size_t)e.first * m + k] = e.second;
        for (long long i = 0; i < n; ++i)
            for (long long j = std::max(0LL, i - bw); j <= i; ++j) {
                double s = 0.0;
                for (int k = 0; k < m; ++k) s += Bd[(size_t)i * m + k] / sigma[k] * Bd[(size_t)j * m + k];
                band[(size_t)(i * W + (j - i + bw))] += s;
            }
    }
    if (!chol_band_factor(band, n, bw)) return fail(h, MGMC_E_INVALID, "coarse precision is not positive definite");
    if (h->chol_G) hipFree(h->chol_G);
    if (h->chol_Li) hipFree(h->chol_Li);
    if (h->chol_blk) hipFree(h->chol_blk);
    h->chol_G = h->chol_Li = h->chol_blk = nullptr;
    h->chol_n = h->chol_B = h->chol_nb = 0;
    if (blocked) {
        std::vector<double> blk[4];
        chol_blocks_host(band, n, bw, B, blk[0], blk[1], blk[2], blk[3]);
        const size_t bytes = blk[0].size() * sizeof(double);
        if (hipMalloc(&h->chol_blk, 4 * bytes) != hipSuccess) {
            h->chol_blk = nullptr;
            return fail(h, MGMC_E_NOMEM, "device allocation failed (blocked coarse Cholesky factors)");
        }
        for (int q = 0; q < 4; ++q)
            HIPCHK(h, hipMemcpy(h->chol_blk + q * blk[0].size(), blk[q].data(), bytes, hipMemcpyHostToDevice));
        h->chol_B = (int)B;
        h->chol_nb = (int)((n + B - 1) / B);
        h->chol_n = (int)n;
        return MGMC_OK;
    }
    std::vector<double> Lm((size_t)n * n, 0.0);
    for (long long i = 0; i < n; ++i)
        for (long long c = std::max(0LL, i - bw); c <= i; ++c) Lm[(size_t)i * n + c] = band[(size_t)(i * W + (c - i + bw))];
    std::vector<double>().swap(band);
    std::vector<double> Li, G;
    chol_inverses_host(Lm, n, Li, G);
    const size_t bytes = (size_t)n * n * sizeof(double);
    if (hipMalloc(&h->chol_G, bytes) != hipSuccess || hipMalloc(&h->chol_Li, bytes) != hipSuccess)
        return fail(h, MGMC_E_NOMEM, "device allocation failed (coarse Cholesky factors)");
    HIPCHK(h, hipMemcpy(h->chol_G, G.data(), bytes, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy(h->chol_Li, Li.data(), bytes, hipMemcpyHostToDevice));
    h->chol_n = (int)n;
    return MGMC_OK;
}

}  // namespace mgmc_host
