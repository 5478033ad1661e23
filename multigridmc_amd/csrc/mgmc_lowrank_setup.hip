// mgmc_lowrank_setup.hip -- the low-rank posterior part: B, Sigma and every level's B_bar on the device (mgmc_set_lowrank;
// measured_operator.cc:9-49, sor_smoother.cc:17-37, linear_operator.cc:10-23 for B_c = R B).
#include "mgmc_internal.hpp"

// ---------------- low-rank posterior part ----------------
namespace {

long long ref_to_layout(const Level& lv, const Layout& L, long long row) {
    const long long nxi = lv.L.nx - 1, nyi = lv.L.ny - 1;
    const int i = (int)(row % nxi) + 1;
    const long long r = row / nxi;
    const int j = (int)(r % nyi) + 1;
    const int k = lv.spec.dim == 3 ? (int)(r / nyi) + 1 : 0;
    return L.at(i, j, k);
}
long long ref_to_padded(const Level& lv, long long row) { return ref_to_layout(lv, lv.L, row); }
int ref_to_tail(const Level& lv, long long row) { return (int)ref_to_layout(lv, tail_layout(lv.L), row); }

template <class T>
int lr_to_device(mgmc_handle* h, LowRankDev& r, T** dst, const std::vector<T>& src) {
    *dst = nullptr;
    if (src.empty()) return MGMC_OK;
    if (hipMalloc((void**)dst, src.size() * sizeof(T)) != hipSuccess) {
        *dst = nullptr;
        return fail(h, MGMC_E_NOMEM, "device allocation failed (low-rank part)");
    }
    r.allocs.push_back(*dst);
    HIPCHK(h, hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
    return MGMC_OK;
}

// B_c = R B, column by column on the device restriction kernel (bitwise the oracle's restrict_)
int lr_restrict_columns(mgmc_handle* h, int level, std::vector<LRColumn>& cols) {
    Level& lf = h->levels[level];
    Level& lc = h->levels[level + 1];
    int rc;
    if ((rc = ensure_scratch(h, level)) || (rc = ensure_scratch(h, level + 1))) return rc;
    std::vector<double> fine(lf.spec.ndof), coarse(lc.spec.ndof);
    for (auto& col : cols) {
        std::fill(fine.begin(), fine.end(), 0.0);
        for (const auto& e : col.ent) fine[e.first] = e.second;
        if ((rc = upload(h, level, fine.data(), lf.scratch[0]))) return rc;
        dim3 block(64, 4, 1);
        dim3 grid = grid3(lc.L.nx - 1, lc.L.ny - 1, lf.spec.dim == 3 ? lc.L.nz - 1 : 1, block);
        if (lf.spec.dim == 3)
            hipLaunchKernelGGL((k_restrict<3>), grid, block, 0, h->stream, lf.L, lc.L, (const double*)lf.scratch[0],
                               lc.scratch[0]);
        else
            hipLaunchKernelGGL((k_restrict<2>), grid, block, 0, h->stream, lf.L, lc.L, (const double*)lf.scratch[0],
                               lc.scratch[0]);
        HIPCHK(h, hipGetLastError());
        if ((rc = download(h, level + 1, lc.scratch[0], coarse.data()))) return rc;
        col.ent.clear();
        for (long long i = 0; i < (long long)coarse.size(); ++i)
            if (col.dense || coarse[i] != 0.0) col.ent.push_back({i, coarse[i]});
    }
    return MGMC_OK;
}

// device data of one level: columns, rows of B, and B_bar for both sweep directions
// (sor_smoother.cc:17-37 with the multicolour splitting: Y = one noise-free multicolour sweep
// from zero per column, M = Sigma + B^T Y, B_bar = Y M^{-1} on the rows where Y is nonzero)
int lr_setup_level(mgmc_handle* h, int level, const std::vector<LRColumn>& cols, const double* sigma, int m) {
    Level& lv = h->levels[level];
    LowRankDev& r = lv.lr;
    r.m = m;
    const long long N = (long long)lv.spec.ndof;
    int rc;
    // columns: entry lists (sparse) or padded value arrays (dense), dot-product blocks
    std::vector<LRColMeta> meta(m);
    std::vector<int> blk_col;
    std::vector<long long> ent_off;
    std::vector<int> t_ent_off;
    std::vector<double> ent_val;
    int ndense = 0;
    // a dense column of a level with at most LR_BLK vertices is one block either way: it is kept as
    // an entry list (every row, ascending: the dense order), so the level can take the small-level
    // kernels (k_lr_small, k_tail)
    std::vector<char> dense_here(m);
    for (int k = 0; k < m; ++k) dense_here[k] = cols[k].dense && N > LR_BLK;
    for (int k = 0; k < m; ++k) {
        const LRColumn& c = cols[k];
        LRColMeta& mt = meta[k];
        mt.n = (long long)c.ent.size();
        r.max_col_n = std::max(r.max_col_n, mt.n);
        mt.blk0 = (int)blk_col.size();
        mt.nblk = (int)((mt.n + LR_BLK - 1) / LR_BLK);
        mt.cflag = 0;
        mt.cval = 0.0;
        for (int b = 0; b < mt.nblk; ++b) blk_col.push_back(k);
        if (dense_here[k]) {
            mt.dense = ndense++;
            mt.ent0 = 0;
        } else {
            mt.dense = -1;
            mt.ent0 = (long long)ent_off.size();
            for (const auto& e : c.ent) {
                ent_off.push_back(ref_to_padded(lv, e.first));
                t_ent_off.push_back(ref_to_tail(lv, e.first));
                ent_val.push_back(e.second);
            }
        }
    }
    // a dense column whose every value is one number (bit for bit; the global average on the fine
    // level, B_g = cell volume: measured_operator.cc:31-45) is read as that constant: no value array is
    // streamed by the dots and the right-hand-side patches (8 bytes per vertex and launch)
    for (int k = 0; k < m; ++k) {
        if (!dense_here[k] || cols[k].ent.empty()) continue;
        uint64_t b0;
        memcpy(&b0, &cols[k].ent[0].second, 8);
        bool same = true;
        for (long long i = 0; i < N && same; ++i) {
            uint64_t bi;
            memcpy(&bi, &cols[k].ent[i].second, 8);
            same = bi == b0;
        }
        if (same) {
            meta[k].cflag = 1;
            meta[k].cval = cols[k].ent[0].second;
        }
    }
    r.nblk = (int)blk_col.size();
    std::vector<LRBlock> blocks(blk_col.size());
    for (int k = 0; k < m; ++k)
        for (int b = 0; b < meta[k].nblk; ++b) {
            LRBlock& B = blocks[(size_t)meta[k].blk0 + b];
            B.e0 = (long long)b * LR_BLK;
            B.cnt = (int)std::min<long long>(LR_BLK, meta[k].n - B.e0);
            B.ent0 = meta[k].dense >= 0 ? 0 : meta[k].ent0 + B.e0;
            B.k = k;
            B.dense = meta[k].dense;
            B.cflag = meta[k].cflag;
            B.cval = meta[k].cval;
            B.sc[0] = 1.0;
            B.sc[1] = 1.0 / sigma[k];  // (the sc_inv values below)
        }
    if ((rc = lr_to_device(h, r, &r.blk, blocks))) return rc;
    if ((rc = lr_to_device(h, r, &r.meta, meta)) || (rc = lr_to_device(h, r, &r.blk_col, blk_col)) ||
        (rc = lr_to_device(h, r, &r.ent_off, ent_off)) || (rc = lr_to_device(h, r, &r.ent_val, ent_val)) ||
        (rc = lr_to_device(h, r, &r.t_ent_off, t_ent_off)))
        return rc;
    if (ndense > 0) {
        const size_t bytes = (size_t)ndense * lv.L.nstore * sizeof(double);
        if (hipMalloc(&r.dense_val, bytes) != hipSuccess) return fail(h, MGMC_E_NOMEM, "device allocation failed");
        r.allocs.push_back(r.dense_val);
        HIPCHK(h, hipMemsetAsync(r.dense_val, 0, bytes, h->stream));
        std::vector<double> v(N);
        for (int k = 0; k < m; ++k) {
            if (!dense_here[k]) continue;
            for (long long i = 0; i < N; ++i) v[i] = cols[k].ent[i].second;
            if ((rc = upload(h, level, v.data(), r.dense_val + (size_t)meta[k].dense * lv.L.nstore))) return rc;
            HIPCHK(h, hipStreamSynchronize(h->stream));
        }
    }
    // dense-column path: exactly one dense column (mgmc_lowrank.hpp k_lr_dense_*)
    r.dense_path = ndense == 1 && !(h->paths & PATH_NO_LR_DENSE);
    r.dense_g = -1;
    for (int k = 0; k < m; ++k)
        if (dense_here[k]) r.dense_g = k;
    r.dense_const = r.dense_g >= 0 && meta[r.dense_g].cflag != 0;
    r.split_g = ndense == 1 && r.dense_const ? r.dense_g : -1;  // (any path: the row lists too)
    r.dense_cval = r.dense_g >= 0 ? meta[r.dense_g].cval : 0.0;
    r.dense_slot = r.dense_g >= 0 ? meta[r.dense_g].dense : 0;
    const int g = r.dense_path ? r.dense_g : -1;
    // bit p of a skip mask over the padded store: set unless p is an interior vertex of `dense_only`
    auto skip_mask = [&](const std::vector<char>& local, uint32_t** dst) {
        std::vector<uint32_t> words((size_t)(lv.L.nstore + 31) / 32, 0xFFFFFFFFu);
        for (long long i = 0; i < N; ++i)
            if (!local[i]) {
                const long long p = ref_to_padded(lv, i);
                words[p >> 5] &= ~(1u << (p & 31));
            }
        return lr_to_device(h, r, dst, words);
    };
    // rows of B (ascending), with the row's coefficients of every column (dense-column path: the
    // rows with an entry in a column other than g)
    std::vector<int> slot(N, -1);
    for (int k = 0; k < m; ++k)
        if (k != g)
            for (const auto& e : cols[k].ent) slot[e.first] = 0;
    if (g >= 0) {
        std::vector<char> local(N);
        for (long long i = 0; i < N; ++i) local[i] = slot[i] == 0;
        if ((rc = skip_mask(local, &r.skip_b))) return rc;
        const size_t fb = (size_t)lv.L.nstore * h->nchains * sizeof(double);
        for (double** q : {&r.fe, &r.fe2}) {
            if (hipMalloc(q, fb) != hipSuccess) return fail(h, MGMC_E_NOMEM, "device allocation failed");
            r.allocs.push_back(*q);
            HIPCHK(h, hipMemsetAsync(*q, 0, fb, h->stream));
        }
        // the fine z-sweep level's kernels read the patched right-hand side in place (k_zsweep_rb7 /
        // k_zresrestrict LRF) when B_g is one number
        r.rhs_inplace = r.dense_path && r.split_g >= 0 && lv.zsweep && level + 1 < (int)h->levels.size() &&
                        zres_lrf_capable(lv, h->levels[level + 1]);
        if (r.rhs_inplace) {
            std::vector<double> ez((size_t)2 * h->nchains, 0.0);
            if ((rc = lr_to_device(h, r, &r.rhs_e, ez))) return rc;
        }
    }
    int nrows = 0;
    std::vector<long long> rows_off;
    std::vector<int> t_rows_off;
    for (long long i = 0; i < N; ++i)
        if (slot[i] == 0) {
            slot[i] = nrows++;
            rows_off.push_back(ref_to_padded(lv, i));
            t_rows_off.push_back(ref_to_tail(lv, i));
        }
    std::vector<double> coef((size_t)nrows * m, 0.0);
    std::vector<uint64_t> mask(nrows, 0);
    for (int k = 0; k < m; ++k)
        for (const auto& e : cols[k].ent) {
            const int u = slot[e.first];
            if (u < 0) continue;  // a dense-only row (dense-column path)
            coef[(size_t)u * m + k] = e.second;
            mask[u] |= 1ull << k;
        }
    r.nrows = nrows;
    // per-chain scratch of a batch: saved f (nrows), dot partials (nblk) and dots (m) per chain
    std::vector<double> sc_one(m, 1.0), sc_inv(m), sq(m), zeros((size_t)std::max(nrows, 1) * h->nchains, 0.0);
    for (int k = 0; k < m; ++k) {
        sc_inv[k] = 1.0 / sigma[k];
        sq[k] = sqrt(1.0 / sigma[k]);  // Sigma^{-1/2} (sor_sampler.cc:30-33)
    }
    if ((rc = lr_to_device(h, r, &r.rows_off, rows_off)) || (rc = lr_to_device(h, r, &r.rows_coef, coef)) ||
        (rc = lr_to_device(h, r, &r.rows_mask, mask)) || (rc = lr_to_device(h, r, &r.save, zeros)) ||
        (rc = lr_to_device(h, r, &r.sc_one, sc_one)) || (rc = lr_to_device(h, r, &r.sc_inv, sc_inv)) ||
        (rc = lr_to_device(h, r, &r.sq, sq)) || (rc = lr_to_device(h, r, &r.t_rows_off, t_rows_off)))
        return rc;
    std::vector<double> partz((size_t)std::max(r.nblk, 1) * h->nchains, 0.0), wz((size_t)m * h->nchains, 0.0);
    if ((rc = lr_to_device(h, r, &r.part, partz)) || (rc = lr_to_device(h, r, &r.w, wz))) return rc;

    // B_bar for the forward and backward splittings
    if ((rc = ensure_scratch(h, level))) return rc;
    std::vector<double> Y((size_t)N * m), b(N), y(N), col(N);
    for (int d = 0; d < 2; ++d) {
        const int direction = d == 0 ? MGMC_FORWARD : MGMC_BACKWARD;
        for (int l = 0; l < m; ++l) {
            std::fill(b.begin(), b.end(), 0.0);
            for (const auto& e : cols[l].ent) b[e.first] = e.second;
            if ((rc = upload(h, level, b.data(), lv.scratch[0]))) return rc;
            HIPCHK(h, hipMemsetAsync(lv.scratch[1], 0, lv.L.nstore * sizeof(double), h->stream));
            GibbsArg g = make_gibbs(h, lv, 0, 0, h->ctrl + 3);
            launch_sweep(lv, lv.scratch[1], lv.scratch[0], g, direction, false, h->stream);
            HIPCHK(h, hipGetLastError());
            if ((rc = download(h, level, lv.scratch[1], y.data()))) return rc;
            for (long long i = 0; i < N; ++i) Y[(size_t)i * m + l] = y[i];
        }
        std::vector<double> M((size_t)m * m), Minv;
        for (int l = 0; l < m; ++l) {
            for (long long i = 0; i < N; ++i) col[i] = Y[(size_t)i * m + l];
            for (int k = 0; k < m; ++k)
                M[(size_t)k * m + l] = (k == l ? sigma[k] : 0.0) + lr_dot_host(cols[k], 1.0, col.data());
        }
        if (!lr_small_inverse(M, m, Minv))
            return fail(h, MGMC_E_INVALID, "Sigma + B^T (L + D/omega)^{-1} B is singular");
        std::vector<long long> boff;
        std::vector<int> t_boff;
        std::vector<double> bval;
        r.nbar_all[d] = 0;
        if (g >= 0) {  // dense-only rows: Y_il = 0 for every l != g; Y_g and row g of Minv on the device
            std::vector<char> local(N);
            for (long long i = 0; i < N; ++i) {
                const double* yi = &Y[(size_t)i * m];
                bool loc = false;
                for (int l = 0; l < m; ++l) loc = loc || (l != g && yi[l] != 0.0);
                local[i] = loc;
                col[i] = yi[g];
                if (!loc && yi[g] != 0.0) ++r.nbar_all[d];
            }
            if ((rc = skip_mask(local, &r.skip_y[d]))) return rc;
            // the table form of Y_g (see LowRankDev::ykey): key = colour parity | neighbour mask << 1,
            // every dense-only vertex of one key must hold the same bits, else Y_g is streamed
            const int dim = lv.spec.dim;
            if (r.dense_const && lv.spec.npoints == 2 * dim + 1 && !lv.field) {
                const int n1 = lv.L.nx - 1, n2 = lv.L.ny - 1, n3 = dim == 3 ? lv.L.nz - 1 : 1;
                std::vector<uint8_t> keys(N);
                std::vector<double> tab(128, 0.0);
                std::vector<char> seen(128, 0);
                bool ok = true;
                for (long long i = 0; i < N && ok; ++i) {
                    const int ii = (int)(i % n1) + 1, jj = (int)((i / n1) % n2) + 1, kk = dim == 3 ? (int)(i / ((long long)n1 * n2)) + 1 : 0;
                    int key = (ii + jj + kk) & 1;
                    key |= (ii > 1 ? 2 : 0) | (ii < n1 ? 4 : 0) | (jj > 1 ? 8 : 0) | (jj < n2 ? 16 : 0);
                    if (dim == 3) key |= (kk > 1 ? 32 : 0) | (kk < n3 ? 64 : 0);
                    keys[i] = (uint8_t)key;
                    if (local[i]) continue;
                    if (!seen[key]) {
                        seen[key] = 1;
                        tab[key] = col[i];
                    } else {
                        ok = memcmp(&tab[key], &col[i], 8) == 0;
                    }
                }
                if (ok) {
                    if (!r.ykey) {  // keys over the padded store (0 elsewhere: masked by skip_y)
                        std::vector<uint8_t> kp((size_t)lv.L.nstore + 16, 0);
                        for (long long i = 0; i < N; ++i) kp[ref_to_padded(lv, i)] = keys[i];
                        if ((rc = lr_to_device(h, r, &r.ykey, kp))) return rc;
                    }
                    if ((rc = lr_to_device(h, r, &r.ytab[d], tab))) return rc;
                }
            }
            const size_t yb = (size_t)lv.L.nstore * sizeof(double);
            if (hipMalloc(&r.yg[d], yb) != hipSuccess) return fail(h, MGMC_E_NOMEM, "device allocation failed");
            r.allocs.push_back(r.yg[d]);
            HIPCHK(h, hipMemsetAsync(r.yg[d], 0, yb, h->stream));
            if ((rc = upload(h, level, col.data(), r.yg[d]))) return rc;
            HIPCHK(h, hipStreamSynchronize(h->stream));
            std::vector<double> mg(Minv.begin() + (size_t)g * m, Minv.begin() + (size_t)(g + 1) * m);
            if ((rc = lr_to_device(h, r, &r.minv_g[d], mg))) return rc;
        }
        for (long long i = 0; i < N; ++i) {
            const double* yi = &Y[(size_t)i * m];
            bool nz = false;
            for (int l = 0; l < m; ++l) nz = nz || ((g < 0 || l != g) && yi[l] != 0.0);
            if (!nz) continue;  // B_bar row is exactly zero: x - 0 = x (dense-column path: a dense-only row)
            boff.push_back(ref_to_padded(lv, i));
            t_boff.push_back(ref_to_tail(lv, i));
            for (int k = 0; k < m; ++k) {
                double u = 0.0;
                for (int l = 0; l < m; ++l) u = std::fma(yi[l], Minv[(size_t)l * m + k], u);
                bval.push_back(u);
            }
        }
        r.nbar[d] = (int)boff.size();
        r.nbar_all[d] += r.nbar[d];
        if ((rc = lr_to_device(h, r, &r.bar_off[d], boff)) || (rc = lr_to_device(h, r, &r.bar_val[d], bval)) ||
            (rc = lr_to_device(h, r, &r.t_bar_off[d], t_boff)))
            return rc;
    }
    bool small = !(h->paths & PATH_NO_LR_SMALL) && ndense == 0 && r.nrows <= (1 << 16) &&
                 r.nbar[0] <= (1 << 16) && r.nbar[1] <= (1 << 16);
    for (int k = 0; k < m; ++k) small = small && meta[k].nblk <= 1;
    r.small = small;
    return MGMC_OK;
}

}  // namespace

extern "C" {

int mgmc_set_lowrank(mgmc_handle* h, int m, const int64_t* colptr, const int64_t* rows, const double* vals,
                     const double* sigma) {
    if (!h) return fail(nullptr, MGMC_E_INVALID, "null handle");
    if (m < 0 || m > LR_MAX_M) return fail(h, MGMC_E_INVALID, "m_lowrank must be in [0, 64]");
    const long long N0 = (long long)h->levels[0].spec.ndof;
    std::vector<LRColumn> cols(m);
    if (m > 0) {
        if (!colptr || !sigma) return fail(h, MGMC_E_INVALID, "null argument");
        if (colptr[0] != 0) return fail(h, MGMC_E_INVALID, "colptr[0] must be 0");
        if (colptr[m] > 0 && (!rows || !vals)) return fail(h, MGMC_E_INVALID, "null argument");
        for (int k = 0; k < m; ++k) {
            if (!(sigma[k] > 0.0) || !std::isfinite(sigma[k])) return fail(h, MGMC_E_INVALID, "Sigma must be positive");
            if (colptr[k + 1] < colptr[k]) return fail(h, MGMC_E_INVALID, "colptr must be non-decreasing");
            for (int64_t q = colptr[k]; q < colptr[k + 1]; ++q) {
                if (rows[q] < 0 || rows[q] >= N0 || (q > colptr[k] && rows[q] <= rows[q - 1]))
                    return fail(h, MGMC_E_INVALID, "row indices of a column must be strictly ascending in [0, N)");
                if (!std::isfinite(vals[q])) return fail(h, MGMC_E_INVALID, "non-finite entry of B");
                cols[k].ent.push_back({rows[q], vals[q]});
            }
            cols[k].dense = (long long)cols[k].ent.size() == N0;
        }
    }
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    destroy_graphs(h);
    for (auto& lv : h->levels) free_lowrank(lv.lr);
    int rc = MGMC_OK;
    for (size_t l = 0; m > 0 && l < h->levels.size(); ++l) {
        if (l > 0 && (rc = lr_restrict_columns(h, (int)l - 1, cols))) break;
        if ((rc = lr_setup_level(h, (int)l, cols, sigma, m))) break;
    }
    if (rc) {
        for (auto& lv : h->levels) free_lowrank(lv.lr);
    }
    h->lr_cols.clear();
    h->lr_sigma.clear();
    if (!rc && m > 0) {
        h->lr_cols = cols;
        h->lr_sigma.assign(sigma, sigma + m);
    }
    if (!rc && h->chol_n > 0)  // the coarse factors carry B_c Sigma^{-1} B_c^T
        rc = build_coarse_chol(h, m > 0 ? &cols : nullptr, sigma, m);
    if (rc) {
        // no half-installed posterior: a failure (a coarse band the blocked Cholesky cannot take, the
        // host work limit, an allocation) leaves the handle with the prior -- no low-rank part on any
        // level and the prior's coarse factors -- and the error code.  The levels' low-rank parts are
        // installed before the coarse factor is built, so they are removed again here.
        const std::string err = h->last_error;
        for (auto& lv : h->levels) free_lowrank(lv.lr);
        h->lr_cols.clear();
        h->lr_sigma.clear();
        h->last_error = err;
        if (h->chol_n > 0 && build_coarse_chol(h, nullptr, nullptr, 0) != MGMC_OK) {
            // the prior's factor built at mgmc_create cannot be rebuilt (e.g. an allocation): no
            // sample call may run on a half-built coarse factor
            h->unusable = true;
            h->last_error = err + "; restoring the prior's coarse Cholesky factor failed too (" + h->last_error +
                            "): the handle is unusable";
        }
        set_global_error(err);
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));
    build_ops(h);
    int rc2 = build_tails(h);
    if (!rc2) rc2 = build_graphs(h);
    if (!rc && !rc2) h->unusable = false;  // a later successful install rebuilt a whole coarse factor
    return rc ? rc : rc2;
}

int mgmc_debug_fail_coarse_factor(mgmc_handle* h, int n) {
    if (!h || n < 0) return fail(h, MGMC_E_INVALID, "invalid argument");
    h->debug_fail_chol = n;
    return MGMC_OK;
}

int mgmc_lowrank_info(const mgmc_handle* h, int level, int direction, int* m, int64_t* nrows_bbar) {
    if (!h || !m || !nrows_bbar) return fail(nullptr, MGMC_E_INVALID, "null argument");
    if (level < 0 || level >= (int)h->levels.size()) return fail(nullptr, MGMC_E_INVALID, "level out of range");
    if (direction != MGMC_FORWARD && direction != MGMC_BACKWARD) return fail(nullptr, MGMC_E_INVALID, "invalid direction");
    const LowRankDev& r = h->levels[level].lr;
    *m = r.m;
    *nrows_bbar = r.nbar_all[direction == MGMC_FORWARD ? 0 : 1];  // local + dense-only rows
    return MGMC_OK;
}

}  // extern "C"
