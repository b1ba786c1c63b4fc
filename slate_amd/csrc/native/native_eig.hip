// Hermitian eigensolver and SVD of the native (Python-free) library:
//   heev = he2hb (stage 1) -> hb2st (stage 2, GPU bulge chase) ->
//          divide & conquer on the real tridiagonal (GPU leaves / merges) ->
//          back-transforms unmtr_hb2st, unmtr_he2hb
//   svd  = ge2tb (stage 1) -> tb2bd (stage 2, GPU bulge chase) -> bdsqr
//          (host implicit QR) -> back-transforms unmbr_tb2bd, unmbr_ge2tb
// (reference src/heev.cc:66-225, src/he2hb.cc, src/hb2st.cc:139-279,
// src/stedc_solve.cc:79-238, src/unmtr_hb2st.cc, src/unmtr_he2hb.cc,
// src/svd.cc:155-364, src/ge2tb.cc, src/tb2bd.cc, src/bdsqr.cc).
//
// MI355X design: the matrix is gathered onto ONE GPU (rank 0; 288 GB of HBM
// holds n = 100k+ in fp64) and every stage runs there on the hand-written
// kernels the Python package uses (geqrf.hip, hb2st.hip, stedc.hip, eig.hip,
// the MFMA GEMM); the eigenvectors go back to the 2D block-cyclic Z in one
// batched point-to-point exchange, the eigenvalues to every rank.  Stage 1
// is GEMM-bound (4/3 n^3 flops): one GPU at 60+ TF/s beats a 2D-distributed
// he2hb's broadcast chain at the sizes the eigensolver is used for (SLATE
// itself runs stage 2 and the tridiagonal solver on one node).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <type_traits>
#include <vector>

#include "../include/bdsqr.hpp"
#include "../include/steqr.hpp"
#include "native_rt.hpp"

namespace slate_amd {
namespace native {

namespace {

// ---------------------------------------------------------------- helpers
template <typename T>
__global__ void real_to_phase_kernel(i64 n, i64 nc, const double* Q, i64 ldq, const T* ph, T* Z, i64 ldz) {
    const i64 i = (i64)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    for (i64 j = blockIdx.y; j < nc; j += gridDim.y) {
        const double q = Q[i + j * ldq];
        if constexpr (slate_hip::scalar_traits<T>::is_complex) {
            const T p = ph ? ph[i] : T{1, 0};
            Z[i + j * ldz] = T{(decltype(p.re))(p.re * q), (decltype(p.re))(p.im * q)};
        } else {
            Z[i + j * ldz] = (T)q;
        }
    }
}

// Z (n x nc, type T) = diag(ph) Q (real); ph: device phases (complex T) or null
template <typename T>
void real_to_phase(i64 n, i64 nc, const double* Q, i64 ldq, const K<T>* ph, K<T>* Z, i64 ldz, hipStream_t s) {
    if (n <= 0 || nc <= 0) return;
    dim3 g((unsigned)((n + 255) / 256), (unsigned)std::min<i64>(nc, 4096));
    hipLaunchKernelGGL(real_to_phase_kernel<K<T>>, g, dim3(256), 0, s, n, nc, Q, ldq, ph, Z, ldz);
    NHIP(hipGetLastError());
}

template <typename V>
Scratch* upload_vec(std::vector<std::unique_ptr<Scratch>>& keep, const std::vector<V>& v, hipStream_t s) {
    keep.push_back(std::make_unique<Scratch>(std::max<size_t>(v.size(), 1) * sizeof(V), s));
    if (!v.empty()) upload(keep.back()->p, v.data(), v.size() * sizeof(V), s);
    return keep.back().get();
}

template <typename V>
std::vector<V> download_vec(const void* d, size_t n, hipStream_t s) {
    std::vector<V> h(n);
    if (n) {
        NHIP(hipMemcpyAsync(h.data(), d, n * sizeof(V), hipMemcpyDeviceToHost, s));
        NHIP(hipStreamSynchronize(s));
    }
    return h;
}

std::vector<i64> argsort(const std::vector<double>& v) {
    std::vector<i64> o(v.size());
    std::iota(o.begin(), o.end(), 0);
    std::stable_sort(o.begin(), o.end(), [&](i64 a, i64 b) { return v[a] < v[b]; });
    return o;
}

// ---------------------------------------------------------------- D & C
// Real symmetric tridiagonal (d, e) of order n -> ascending eigenvalues w
// (host) and the eigenvectors Q (device, n x n, ld n), one process:
// leaves of <= 128 rows solved all at once on the GPU (steqr_leaves), then
// every merge of the split-at-the-middle tree bottom-up (LAPACK laed1-4 /
// the reference's stedc_merge / deflate / secular / z_vector): host
// deflation and Givens chains on O(s) vectors, device rotations, secular
// roots, rank-one vectors and laed3's split GEMM (models/stedc.py _merge).
struct Merge { i64 a, m, b; };

void dc_tree(i64 a, i64 b, int t, i64 leaf, std::vector<std::pair<i64, i64>>& leaves,
             std::vector<std::vector<Merge>>& levels) {
    if (b - a <= leaf) {
        leaves.push_back({a, b});
        return;
    }
    const i64 m = a + (b - a) / 2;
    if ((int)levels.size() <= t) levels.resize(t + 1);
    levels[t].push_back({a, m, b});
    dc_tree(a, m, t + 1, leaf, leaves, levels);
    dc_tree(m, b, t + 1, leaf, leaves, levels);
}

// One merge on the rows [r0, r1) of the eigenvector matrix that this process
// holds (Q: those rows of every column, ld ldq; the whole matrix for one
// process).  z = [last row of the top child's vectors, first row of the
// bottom child's] (host, b - a entries, identical on every rank), so the
// host deflation / secular logic gives the same eigenvalues everywhere and
// each rank updates only its rows: permutations, rotations and laed3's split
// GEMM act on nr = |[a, b) n [r0, r1)| rows (models/stedc.py _merge).
void dc_merge_rows(const Merge& g, double rho, std::vector<double>& w, const std::vector<double>& z, double* Q,
                   i64 ldq, i64 r0, i64 r1, hipStream_t s) {
    const i64 a = g.a, m = g.m, b = g.b, S = b - a;
    const i64 lo = std::max(a, r0), hi = std::min(b, r1), nr = std::max<i64>(hi - lo, 0);
    const i64 split = std::min(std::max<i64>(m - lo, 0), nr);     // local rows [0, split) are the top child's
    std::vector<std::unique_ptr<Scratch>> keep;
    std::vector<double> dd(w.begin() + a, w.begin() + b);
    double* Qm = Q + (lo - r0) + a * ldq;          // my rows of the merge's columns
    const i64 lds = std::max<i64>(nr, 1);
    Scratch Qs((size_t)lds * S * sizeof(double), s);
    double* qs = Qs.as<double>();
    auto permute_cols = [&](const std::vector<i64>& o, const double* src, i64 ld_src, double* dst, i64 ld_dst) {
        if (!nr) return;
        Scratch* id = upload_vec(keep, o, s);
        slate_hip::cols_copy(nr, S, src, ld_src, id->as<i64>(), dst, ld_dst, false, s);
    };
    if (rho == 0.0) {
        const std::vector<i64> o = argsort(dd);
        permute_cols(o, Qm, ldq, qs, lds);
        if (nr) copy2d(Qm, ldq, qs, lds, nr, S, s);
        for (i64 i = 0; i < S; ++i) w[a + i] = dd[o[i]];
        NHIP(hipStreamSynchronize(s));
        return;
    }
    const bool flip = rho < 0;
    if (flip) {
        for (auto& x : dd) x = -x;
        rho = -rho;
    }
    // ---- sort the poles ascending; column types 1 = top child, 2 = bottom
    const std::vector<i64> order = argsort(dd);
    std::vector<double> d2((size_t)S), z2((size_t)S);
    std::vector<int> ty((size_t)S);
    for (i64 i = 0; i < S; ++i) {
        d2[i] = dd[order[i]];
        z2[i] = z[order[i]];
        ty[i] = order[i] < (m - a) ? 1 : 2;
    }
    permute_cols(order, Qm, ldq, qs, lds);
    // ---- deflation: tiny z components, then Givens chains over close poles
    const double eps = std::numeric_limits<double>::epsilon();
    double zz = 0, dmax = 0;
    for (i64 i = 0; i < S; ++i) { zz += z2[i] * z2[i]; dmax = std::max(dmax, std::abs(d2[i])); }
    const double tolf = 8.0 * eps * std::max(dmax, rho * zz);
    std::vector<i64> c;
    for (i64 i = 0; i < S; ++i)
        if (!(rho * std::abs(z2[i]) * std::sqrt(zz) <= tolf)) c.push_back(i);
    std::vector<i64> Kidx;
    if (!c.empty()) {
        const i64 nn = (i64)c.size();
        std::vector<double> cs((size_t)nn, 0.0), sn((size_t)nn, 0.0);
        std::vector<int> rot((size_t)nn, 0), kp((size_t)nn, 1);
        std::vector<i64> rI, rJ;
        std::vector<double> rC, rS;
        i64 t = 0;
        while (t < nn) {
            double acc = z2[c[t]];
            int tacc = ty[c[t]];
            i64 u = t + 1;
            while (u < nn && d2[c[u]] - d2[c[u - 1]] <= tolf) {
                const double bb = z2[c[u]];
                const double r = std::hypot(acc, bb);
                cs[u] = r == 0 ? 1.0 : bb / r;
                sn[u] = r == 0 ? 0.0 : acc / r;
                rot[u] = 1;
                z2[c[u - 1]] = 0.0;
                z2[c[u]] = r;
                tacc |= ty[c[u]];
                ty[c[u]] = tacc;
                kp[u - 1] = 0;
                rI.push_back(c[u - 1]);
                rJ.push_back(c[u]);
                rC.push_back(cs[u]);
                rS.push_back(sn[u]);
                acc = r;
                ++u;
            }
            kp[u - 1] = 1;
            t = u;
        }
        if (!rI.empty() && nr) {
            Scratch* I = upload_vec(keep, rI, s);
            Scratch* J = upload_vec(keep, rJ, s);
            Scratch* C = upload_vec(keep, rC, s);
            Scratch* Sn = upload_vec(keep, rS, s);
            slate_hip::rot_cols(nr, qs, lds, (i64)rI.size(), I->as<i64>(), J->as<i64>(), C->as<double>(),
                                Sn->as<double>(), s);
        }
        for (i64 u = 0; u < nn; ++u)
            if (kp[u]) Kidx.push_back(c[u]);
    }
    std::vector<double> lam = d2;
    const i64 k = (i64)Kidx.size();
    if (k) {
        std::vector<double> dK((size_t)k), zK((size_t)k);
        double zzK = 0;
        for (i64 i = 0; i < k; ++i) { dK[i] = d2[Kidx[i]]; zK[i] = z2[Kidx[i]]; zzK += zK[i] * zK[i]; }
        Scratch* dKd = upload_vec(keep, dK, s);
        Scratch* zKd = upload_vec(keep, zK, s);
        Scratch org((size_t)k * sizeof(i64), s), mu((size_t)k * sizeof(double), s), zh((size_t)k * sizeof(double), s);
        slate_hip::stedc_secular(k, dKd->as<double>(), zKd->as<double>(), rho, zzK, org.as<i64>(), mu.as<double>(),
                                 zh.as<double>(), nullptr, 0, s);
        const std::vector<i64> orgh = download_vec<i64>(org.p, (size_t)k, s);
        const std::vector<double> muh = download_vec<double>(mu.p, (size_t)k, s);
        for (i64 i = 0; i < k; ++i) lam[Kidx[i]] = dK[orgh[i]] + muh[i];
        // ---- Qs[:, K] <- Qs[:, K] V: the top rows meet only the K columns
        // of type 1 | 3, the bottom rows only those of type 2 | 3
        struct Part { i64 r0, r1; std::vector<i64> sel; };
        std::vector<Part> parts;
        parts.push_back({0, split, {}});
        parts.push_back({split, nr, {}});
        for (i64 i = 0; i < k; ++i) {
            if (ty[Kidx[i]] & 1) parts[0].sel.push_back(i);
            if (ty[Kidx[i]] & 2) parts[1].sel.push_back(i);
        }
        if (nr) {
            Scratch* Kd = upload_vec(keep, Kidx, s);
            std::vector<std::unique_ptr<Scratch>> srcs;
            std::vector<Scratch*> seld;
            for (auto& pt : parts) {
                const i64 np = pt.r1 - pt.r0, ns = (i64)pt.sel.size();
                if (!ns || !np) { srcs.push_back(nullptr); seld.push_back(nullptr); continue; }
                std::vector<i64> cols((size_t)ns);
                for (i64 i = 0; i < ns; ++i) cols[i] = Kidx[pt.sel[i]];
                Scratch* cd = upload_vec(keep, cols, s);
                srcs.push_back(std::make_unique<Scratch>((size_t)np * ns * sizeof(double), s));
                slate_hip::cols_copy(np, ns, qs + pt.r0, lds, cd->as<i64>(), srcs.back()->as<double>(), np, false, s);
                seld.push_back(upload_vec(keep, pt.sel, s));
            }
            // rank-one vector columns per chunk: at most ~the merge block's
            // size (a row-distributed merge holds only nr of the S rows)
            static const i64 chdiv = [] { const char* e = std::getenv("SLATE_AMD_DC_CHDIV"); return e ? std::atoll(e) : 4; }();
            const i64 CH = chdiv <= 0 ? 4096
                                      : std::max<i64>(256, std::min<i64>(4096, (nr * S) / (chdiv * std::max<i64>(k, 1))));
            for (i64 j0 = 0; j0 < k; j0 += CH) {
                const i64 nc = std::min(CH, k - j0);
                Scratch V((size_t)k * nc * sizeof(double), s);
                slate_hip::stedc_vectors(k, dKd->as<double>(), zh.as<double>(), org.as<i64>(), mu.as<double>(), j0,
                                         nc, V.as<double>(), k, s);
                for (size_t pi = 0; pi < parts.size(); ++pi) {
                    const Part& pt = parts[pi];
                    const i64 np = pt.r1 - pt.r0, ns = (i64)pt.sel.size();
                    if (!np) continue;
                    Scratch out((size_t)np * nc * sizeof(double), s);
                    if (ns) {
                        Scratch Vp((size_t)ns * nc * sizeof(double), s);
                        slate_hip::permute_rows_gather<double>(ns, nc, V.as<double>(), k, Vp.as<double>(), ns,
                                                               seld[pi]->as<i64>(), s);
                        gemm_k<double>('N', 'N', np, nc, ns, 1.0, srcs[pi]->as<double>(), np, Vp.as<double>(), ns,
                                       0.0, out.as<double>(), np, s);
                    } else {
                        dzero(out.p, (size_t)np * nc * sizeof(double), s);
                    }
                    slate_hip::cols_copy(np, nc, out.as<double>(), np, Kd->as<i64>() + j0, qs + pt.r0, lds, true, s);
                }
            }
        }
    }
    if (flip)
        for (auto& x : lam) x = -x;
    const std::vector<i64> o2 = argsort(lam);
    for (i64 i = 0; i < S; ++i) w[a + i] = lam[o2[i]];
    if (nr) {
        Scratch* od = upload_vec(keep, o2, s);
        slate_hip::cols_copy(nr, S, qs, lds, od->as<i64>(), Qm, ldq, false, s);
    }
    NHIP(hipStreamSynchronize(s));
}

// One tree LEVEL of merges with the sort, deflation, close-pole rotations
// and every index set formed on the device (stedc_level_prep), ONE host read
// of the per-merge sizes, then per merge the rotations, the secular solve,
// laed3's split GEMM and the final ordering -- models/stedc.py
// _merge_level_gpu, for one process (all rows).  wd: the device copy of the
// eigenvalues (updated in place), Q: n x n (ld ldq).
struct LevelWork {
    std::vector<std::unique_ptr<Scratch>> keep;
    double *dd, *zs, *cs, *sn, *rC, *rS, *lam;
    int *ty, *kp_, *rot;
    i64 *order, *c, *K, *S1, *KS1, *S2, *KS2, *D, *isK, *rI, *rJ, *o2;
    LevelWork(i64 n, hipStream_t s) {
        const size_t nn = (size_t)std::max<i64>(n, 1);
        auto f = [&](size_t es) { keep.push_back(std::make_unique<Scratch>(nn * es, s)); return keep.back()->p; };
        dd = (double*)f(8); zs = (double*)f(8); cs = (double*)f(8); sn = (double*)f(8); rC = (double*)f(8);
        rS = (double*)f(8); lam = (double*)f(8);
        ty = (int*)f(4); kp_ = (int*)f(4); rot = (int*)f(4);
        order = (i64*)f(8); c = (i64*)f(8); K = (i64*)f(8); S1 = (i64*)f(8); KS1 = (i64*)f(8); S2 = (i64*)f(8);
        KS2 = (i64*)f(8); D = (i64*)f(8); isK = (i64*)f(8); rI = (i64*)f(8); rJ = (i64*)f(8); o2 = (i64*)f(8);
    }
};

void dc_level_device(const std::vector<Merge>& lev, const std::vector<double>& e, LevelWork& ws, const double* W,
                     const double* Z, double* wd, double* Q, i64 ldq, i64 n, hipStream_t s) {
    const i64 nm = (i64)lev.size();
    if (!nm) return;
    std::vector<std::unique_ptr<Scratch>> keep;
    std::vector<i64> desc;
    std::vector<double> rhos;
    i64 maxs = 1;
    for (auto& g : lev) {
        const double r = e[g.m - 1];
        desc.insert(desc.end(), {g.a, g.m, g.b, r < 0 ? 1 : 0});
        rhos.push_back(std::abs(r));
        maxs = std::max(maxs, g.b - g.a);
    }
    Scratch* descd = upload_vec(keep, desc, s);
    Scratch* rhod = upload_vec(keep, rhos, s);
    const size_t mb = slate_hip::stedc_meta_bytes();
    Scratch meta((size_t)nm * mb, s);
    slate_hip::stedc_level_prep(n, nm, maxs, descd->as<i64>(), rhod->as<double>(), W, Z, ws.dd, ws.zs, ws.ty,
                                ws.order, ws.c, ws.kp_, ws.rot, ws.cs, ws.sn, meta.p, ws.K, ws.S1, ws.KS1, ws.S2,
                                ws.KS2, ws.D, ws.isK, ws.rI, ws.rJ, ws.rC, ws.rS, s);
    const std::vector<unsigned char> mh = download_vec<unsigned char>(meta.p, (size_t)nm * mb, s);
    for (i64 t = 0; t < nm; ++t) {
        const Merge& g = lev[(size_t)t];
        const i64 a = g.a, m = g.m, b = g.b, S = b - a;
        i64 ints[8];
        double dbl[2];
        std::memcpy(ints, mh.data() + (size_t)t * mb, sizeof ints);
        std::memcpy(dbl, mh.data() + (size_t)t * mb + 64, sizeof dbl);
        const i64 k = ints[1], nrot = ints[2], n1 = ints[3], n2 = ints[4], nd = ints[5];
        const double zzK = dbl[1];
        const int flip = e[m - 1] < 0 ? 1 : 0;
        const double r = std::abs(e[m - 1]);
        double* qm = Q + a + a * ldq;                          // rows a..b of columns a..b
        Scratch Qs((size_t)S * S * sizeof(double), s);
        slate_hip::cols_copy(S, S, qm, ldq, ws.order + a, Qs.as<double>(), S, false, s);
        if (nrot) slate_hip::rot_cols(S, Qs.as<double>(), S, nrot, ws.rI + a, ws.rJ + a, ws.rC + a, ws.rS + a, s);
        Scratch dK((size_t)std::max<i64>(k, 1) * 8, s), org((size_t)std::max<i64>(k, 1) * 8, s),
            mu((size_t)std::max<i64>(k, 1) * 8, s), zK((size_t)std::max<i64>(k, 1) * 8, s),
            zh((size_t)std::max<i64>(k, 1) * 8, s);
        if (k) {
            slate_hip::vec_gather(k, ws.dd + a, ws.K + a, dK.as<double>(), s);
            slate_hip::vec_gather(k, ws.zs + a, ws.K + a, zK.as<double>(), s);
            slate_hip::stedc_secular(k, dK.as<double>(), zK.as<double>(), r, zzK, org.as<i64>(), mu.as<double>(),
                                     zh.as<double>(), nullptr, 0, s);
        }
        slate_hip::stedc_lambda(S, ws.dd + a, ws.isK + a, dK.as<double>(), org.as<i64>(), mu.as<double>(), flip,
                                ws.lam + a, s);
        if (k) {
            // Qs[:, K] <- Qs[:, K] V: rows above m with the K columns nonzero
            // there (S1 / KS1), rows below with S2 / KS2; V in column chunks
            struct Part { i64 ra, rb, ns; i64 *Sx, *KSx; };
            std::vector<Part> parts{{0, m - a, n1, ws.S1, ws.KS1}, {m - a, S, n2, ws.S2, ws.KS2}};
            std::vector<std::unique_ptr<Scratch>> srcs;
            for (auto& pt : parts) {
                if (!pt.ns || pt.rb <= pt.ra) { srcs.push_back(nullptr); continue; }
                const i64 np = pt.rb - pt.ra;
                srcs.push_back(std::make_unique<Scratch>((size_t)np * pt.ns * 8, s));
                slate_hip::cols_copy(np, pt.ns, Qs.as<double>() + pt.ra, S, pt.KSx + a, srcs.back()->as<double>(), np,
                                     false, s);
            }
            const i64 CH = 4096;
            for (i64 j0 = 0; j0 < k; j0 += CH) {
                const i64 nc = std::min(CH, k - j0);
                Scratch V((size_t)k * nc * 8, s);
                slate_hip::stedc_vectors(k, dK.as<double>(), zh.as<double>(), org.as<i64>(), mu.as<double>(), j0, nc,
                                         V.as<double>(), k, s);
                for (size_t pi = 0; pi < parts.size(); ++pi) {
                    const Part& pt = parts[pi];
                    const i64 np = pt.rb - pt.ra;
                    if (np <= 0) continue;
                    Scratch out((size_t)np * nc * 8, s);
                    if (srcs[pi]) {
                        Scratch Vp((size_t)pt.ns * nc * 8, s);
                        slate_hip::permute_rows_gather<double>(pt.ns, nc, V.as<double>(), k, Vp.as<double>(), pt.ns,
                                                               pt.Sx + a, s);
                        gemm_k<double>('N', 'N', np, nc, pt.ns, 1.0, srcs[pi]->as<double>(), np, Vp.as<double>(),
                                       pt.ns, 0.0, out.as<double>(), np, s);
                    } else {
                        dzero(out.p, (size_t)np * nc * 8, s);
                    }
                    slate_hip::cols_copy(np, nc, out.as<double>(), np, ws.K + a + j0, Qs.as<double>() + pt.ra, S, true,
                                         s);
                }
            }
        }
        slate_hip::stedc_merge2(ws.lam + a, ws.K + a, k, ws.D + a, nd, flip, ws.o2 + a, s);
        slate_hip::vec_gather(S, ws.lam + a, ws.o2 + a, wd + a, s);
        slate_hip::cols_copy(S, S, Qs.as<double>(), S, ws.o2 + a, qm, ldq, false, s);
    }
    NHIP(hipStreamSynchronize(s));
}

// Divide & conquer with the eigenvector matrix distributed by ROWS: this
// process holds rows [r0, r1) of every column (Q, ld ldq), w (all n
// eigenvalues) ends identical on every rank.  Every rank solves every leaf
// (their eigenvalues are needed by all; only its rows of the leaf vectors
// are stored), and per tree level ONE all-reduce of n doubles over `comm`
// assembles the merges' z vectors from the rows' owners (the reference's
// stedc_z_vector.cc:94 MPI_Allreduce).  comm == nullptr: one process, all
// rows (r0 = 0, r1 = n).
void stedc_rows(i64 n, const std::vector<double>& d, const std::vector<double>& e, std::vector<double>& w,
                double* Q, i64 ldq, i64 r0, i64 r1, Comm* comm, hipStream_t s) {
    w.assign((size_t)n, 0.0);
    if (n == 0) return;
    const i64 nr = std::max<i64>(r1 - r0, 0);
    if (nr) dzero(Q, (size_t)ldq * n * sizeof(double), s);
    std::vector<std::pair<i64, i64>> leaves;
    std::vector<std::vector<Merge>> levels;
    dc_tree(0, n, 0, 128, leaves, levels);
    std::vector<double> dl = d;
    for (auto& lev : levels)
        for (auto& g : lev) {
            const double rho = e[g.m - 1];
            dl[g.m - 1] -= rho;
            dl[g.m] -= rho;
        }
    {
        std::vector<std::unique_ptr<Scratch>> keep;
        std::vector<i64> lo, hi;
        i64 mx = 1;
        for (auto& l : leaves) { lo.push_back(l.first); hi.push_back(l.second); mx = std::max(mx, l.second - l.first); }
        std::vector<double> ee(e);
        ee.resize((size_t)n, 0.0);
        Scratch* lod = upload_vec(keep, lo, s);
        Scratch* hid = upload_vec(keep, hi, s);
        Scratch* dd = upload_vec(keep, dl, s);
        Scratch* ed = upload_vec(keep, ee, s);
        Scratch wd((size_t)n * sizeof(double), s), fails(sizeof(i64), s);
        dzero(fails.p, sizeof(i64), s);
        slate_hip::steqr_leaves((i64)leaves.size(), lod->as<i64>(), hid->as<i64>(), dd->as<double>(),
                                ed->as<double>(), wd.as<double>(), Q, ldq, r0, r1, fails.as<i64>(), s, (int)mx, 60);
        w = download_vec<double>(wd.p, (size_t)n, s);
        if (download_vec<i64>(fails.p, 1, s)[0])
            throw Error("native heev: a divide & conquer leaf did not converge");
    }
    Scratch zb((size_t)n * sizeof(double), s);
    // one process, all rows: the level-batched device merges (default;
    // SLATE_AMD_NATIVE_DC_DEVICE=0 keeps the per-merge host logic below)
    static const bool dev_merge = [] { const char* e = std::getenv("SLATE_AMD_NATIVE_DC_DEVICE"); return !(e && e[0] == '0'); }();
    if (dev_merge && !comm && r0 == 0 && r1 == n) {
        LevelWork ws(n, s);
        Scratch wdv((size_t)n * sizeof(double), s), Wl((size_t)n * sizeof(double), s);
        upload(wdv.p, w.data(), (size_t)n * sizeof(double), s);
        for (int t = (int)levels.size() - 1; t >= 0; --t) {
            dzero(zb.p, (size_t)n * sizeof(double), s);
            double* z = zb.as<double>();
            for (auto& g : levels[t]) {
                copy2d(z + g.a, 1, Q + (g.m - 1) + g.a * ldq, ldq, 1, g.m - g.a, s);
                copy2d(z + g.m, 1, Q + g.m + g.m * ldq, ldq, 1, g.b - g.m, s);
            }
            dcopy(Wl.p, wdv.p, (size_t)n * sizeof(double), s);      // the children's eigenvalues of this level
            dc_level_device(levels[t], e, ws, Wl.as<double>(), z, wdv.as<double>(), Q, ldq, n, s);
        }
        w = download_vec<double>(wdv.p, (size_t)n, s);
        return;
    }
    for (int t = (int)levels.size() - 1; t >= 0; --t) {
        // z of every merge of this level from the owners of rows m - 1 and m
        dzero(zb.p, (size_t)n * sizeof(double), s);
        double* z = zb.as<double>();
        for (auto& g : levels[t]) {
            if (g.m - 1 >= r0 && g.m - 1 < r1)
                copy2d(z + g.a, 1, Q + (g.m - 1 - r0) + g.a * ldq, ldq, 1, g.m - g.a, s);
            if (g.m >= r0 && g.m < r1) copy2d(z + g.m, 1, Q + (g.m - r0) + g.m * ldq, ldq, 1, g.b - g.m, s);
        }
        if (comm && comm->size > 1) comm->allreduce(zb.p, (size_t)n, DT::F64, 's', s);
        const std::vector<double> zh = download_vec<double>(zb.p, (size_t)n, s);
        for (auto& g : levels[t])
            dc_merge_rows(g, e[g.m - 1], w, std::vector<double>(zh.begin() + g.a, zh.begin() + g.b), Q, ldq, r0, r1,
                          s);
    }
}

// one process: every row
void stedc_device(i64 n, const std::vector<double>& d, const std::vector<double>& e, std::vector<double>& w,
                  double* Q, i64 ldq, hipStream_t s) {
    stedc_rows(n, d, e, w, Q, ldq, 0, n, nullptr, s);
}

// ---------------------------------------------------------------- stage 1
template <typename T>
struct Panel { i64 r0, kk; std::unique_ptr<Scratch> V, T_; };

// zero the strictly lower part of an m x k block
template <typename T>
void zero_strict_lower(i64 m, i64 k, T* P, i64 ld, hipStream_t s) {
    if (m <= 1 || k <= 0) return;
    slate_hip::TriMask mk;
    mk.mode = 2;
    slate_hip::gecopy_mask<K<T>>(mk, m, k, kp(P), ld, kp(P), ld, false, s);
}

// dense Hermitian Af (n x n, ld n, both triangles) -> band of width nb in
// place; the panel reflectors (explicit V, T) are kept for the back-transform.
// Lookahead (models/eig.py he2hb's pipelining; SLATE_AMD_NATIVE_HE2HB_LOOKAHEAD=0
// disables): the rank-2k update of step k first updates the next panel's
// columns, and that panel's QR runs on the side stream (rt().panel) while the
// bulk of the update streams the rest of A22
template <typename T>
void he2hb(i64 n, i64 nb, T* Af, i64 ld, std::vector<Panel<T>>& panels, hipStream_t s) {
    const char ct = ctrans<T>();
    static const bool la_env = [] { const char* e = std::getenv("SLATE_AMD_NATIVE_HE2HB_LOOKAHEAD"); return !(e && e[0] == '0'); }();
    hipStream_t side = rt().panel;
    const bool la = la_env && side != nullptr && side != s;
    hipEvent_t ev_upd = nullptr, ev_qr = nullptr;
    if (la) {
        NHIP(hipEventCreateWithFlags(&ev_upd, hipEventDisableTiming));
        NHIP(hipEventCreateWithFlags(&ev_qr, hipEventDisableTiming));
    }
    struct EvGuard {
        hipEvent_t a, b;
        ~EvGuard() { if (a) (void)hipEventDestroy(a); if (b) (void)hipEventDestroy(b); }
    } ev_guard{ev_upd, ev_qr};
    // per-call workspaces sized for the first (largest) panel: no allocation
    // inside the panel loop (the loop is launch-bound at the small panels)
    const i64 mmax = std::max<i64>(n - nb, 1);
    Scratch tau((size_t)nb * sizeof(T), s), X((size_t)mmax * nb * sizeof(T), s),
        VW((size_t)mmax * 2 * nb * sizeof(T), s), WV((size_t)mmax * 2 * nb * sizeof(T), s),
        Mt((size_t)nb * nb * sizeof(T), s);
    auto make_panel = [&](i64 k0) {
        const i64 r0 = k0 + nb, kb = std::min(nb, n - k0), m = n - r0;
        Panel<T> pn;
        pn.r0 = r0;
        pn.kk = std::min(m, kb);
        pn.V = std::make_unique<Scratch>((size_t)m * pn.kk * sizeof(T), s);
        pn.T_ = std::make_unique<Scratch>((size_t)pn.kk * pn.kk * sizeof(T), s);
        return pn;
    };
    auto panel_qr = [&](i64 k0, Panel<T>& pn, hipStream_t st) {
        const i64 r0 = k0 + nb, kb = std::min(nb, n - k0), m = n - r0;
        dzero(tau.p, (size_t)pn.kk * sizeof(T), st);
        slate_hip::geqrf_panel_ws<K<T>>(m, kb, kp(Af + r0 + k0 * ld), ld, kp(tau.as<T>()),
                                        kp(pn.T_->template as<T>()), pn.kk, kp(pn.V->template as<T>()), m,
                                        rt().qr_work, st);
    };
    bool have_next = false;      // panels.back() is the next panel, factored on the side stream
    Panel<T> next;
    for (i64 k0 = 0; k0 < n - nb; k0 += nb) {
        const i64 r0 = k0 + nb, kb = std::min(nb, n - k0), m = n - r0;
        if (m <= 0) break;
        const i64 kk = std::min(m, kb);
        T* P = Af + r0 + k0 * ld;
        Panel<T> pn;
        if (have_next) {
            pn = std::move(next);
            NHIP(hipStreamWaitEvent(s, ev_qr, 0));
            have_next = false;
        } else {
            pn = make_panel(k0);
            panel_qr(k0, pn, s);
        }
        T* V = pn.V->template as<T>();
        T* Tm = pn.T_->template as<T>();
        // band part: R, the reflectors zeroed, mirrored to the upper triangle
        zero_strict_lower<T>(m, kb, P, ld, s);
        // (gecopy's m x n are the DESTINATION's: kb x m here)
        slate_hip::gecopy<K<T>, K<T>>('G', ct, kb, m, kp(P), ld, kp(Af + k0 + r0 * ld), ld, s);
        // X = V T, Y = A22 X, M = X^H Y, W = Y - V M / 2, A22 -= V W^H + W V^H
        copy2d(X.as<T>(), m, V, m, m, kk, s);
        slate_hip::trmm<K<T>>('R', 'U', 'N', 'N', m, kk, kv(T(1)), kp(Tm), kk, kp(X.as<T>()), m, s);
        T* Y = VW.as<T>() + m * kk;
        T* A22 = Af + r0 + r0 * ld;
        gemm_k<T>('N', 'N', m, kk, m, T(1), A22, ld, X.as<T>(), m, T(0), Y, m, s);
        gemm_k<T>(ct, 'N', kk, kk, m, T(1), X.as<T>(), m, Y, m, T(0), Mt.as<T>(), kk, s);
        gemm_k<T>('N', 'N', m, kk, kk, T(-0.5), V, m, Mt.as<T>(), kk, T(1), Y, m, s);
        copy2d(VW.as<T>(), m, V, m, m, kk, s);
        copy2d(WV.as<T>(), m, Y, m, m, kk, s);
        copy2d(WV.as<T>() + m * kk, m, V, m, m, kk, s);
        // the next panel: columns r0 .. r0 + kbn of A22, rows r0 + nb ..
        const i64 k1 = r0, kbn = std::min(nb, n - k1), mn = n - (k1 + nb);
        if (la && mn > 0 && kbn < m) {
            gemm_k<T>('N', ct, m, kbn, 2 * kk, T(-1), VW.as<T>(), m, WV.as<T>(), m, T(1), A22, ld, s);
            next = make_panel(k1);                    // allocated on s before the event
            NHIP(hipEventRecord(ev_upd, s));
            NHIP(hipStreamWaitEvent(side, ev_upd, 0));
            panel_qr(k1, next, side);
            NHIP(hipEventRecord(ev_qr, side));
            have_next = true;
            gemm_k<T>('N', ct, m, m - kbn, 2 * kk, T(-1), VW.as<T>(), m, WV.as<T>() + kbn, m, T(1), A22 + kbn * ld,
                      ld, s);
        } else {
            gemm_k<T>('N', ct, m, m, 2 * kk, T(-1), VW.as<T>(), m, WV.as<T>(), m, T(1), A22, ld, s);
        }
        panels.push_back(std::move(pn));
    }
    if (have_next) NHIP(hipStreamWaitEvent(s, ev_qr, 0));     // (not reached: the loop consumes it)
}

// Z := Q1 Z, Q1 = H_0 H_1 ... (panels last to first: Z -= V T (V^H Z)).
// Groups of G = SLATE_AMD_UNMTR_HE2HB_GROUP (default 8 here) consecutive panels
// are merged into ONE block reflector I - Vg Tg Vg^H (forward larft merge,
// Tg = [[T1, -T1 V1^H V2 T2], [0, T2]]): Z streams once per group with
// K = G nb instead of once per panel with K = nb (models/eig.py
// unmtr_he2hb / _merge_reflectors).
template <typename T>
struct QGroup { i64 r0, m, kt; std::unique_ptr<Scratch> Vg, Tg; };

inline i64 unmtr_he2hb_group() {
    static const i64 G = [] { const char* e = std::getenv("SLATE_AMD_UNMTR_HE2HB_GROUP"); return e ? std::max(1, std::atoi(e)) : 8; }();
    return G;
}

// the merged groups, last group first.  The buffers are allocated on
// stream sa (the stream that later applies and frees them); the merge work
// (he2hb_groups_fill) runs on sw, ordered after sa by the event `ready`
template <typename T>
std::vector<QGroup<T>> he2hb_groups(i64 n, std::vector<Panel<T>>& panels, i64 G, hipStream_t sa, hipStream_t sw,
                                    hipEvent_t ready) {
    std::vector<QGroup<T>> gs;
    for (i64 i1 = (i64)panels.size(); i1 > 0;) {
        const i64 i0 = std::max<i64>(0, i1 - G);
        QGroup<T> g;
        g.r0 = panels[i0].r0;
        g.m = n - g.r0;
        g.kt = 0;
        for (i64 i = i0; i < i1; ++i) g.kt += panels[i].kk;
        g.Vg = std::make_unique<Scratch>((size_t)g.m * g.kt * sizeof(T), sa);
        g.Tg = std::make_unique<Scratch>((size_t)g.kt * g.kt * sizeof(T), sa);
        gs.push_back(std::move(g));
        i1 = i0;
    }
    if (sw != sa) {
        NHIP(hipEventRecord(ready, sa));
        NHIP(hipStreamWaitEvent(sw, ready, 0));
    }
    return gs;
}

template <typename T>
void he2hb_groups_fill(i64 n, std::vector<Panel<T>>& panels, i64 G, std::vector<QGroup<T>>& gs, hipStream_t sw) {
    const char ct = ctrans<T>();
    i64 i1 = (i64)panels.size();
    for (auto& g : gs) {
        const i64 i0 = std::max<i64>(0, i1 - G), r0 = g.r0, m = g.m, kt = g.kt;
        T* vg = g.Vg->template as<T>();
        T* tg = g.Tg->template as<T>();
        dzero(vg, (size_t)m * kt * sizeof(T), sw);
        dzero(tg, (size_t)kt * kt * sizeof(T), sw);
        i64 c = 0;
        for (i64 i = i0; i < i1; ++i) {
            const Panel<T>& pn = panels[i];
            const i64 kb = pn.kk, off = pn.r0 - r0, mi = n - pn.r0;
            const T* Vi = pn.V->template as<T>();
            const T* Ti = pn.T_->template as<T>();
            copy2d(vg + off + c * m, m, Vi, mi, mi, kb, sw);
            copy2d(tg + c + c * kt, kt, Ti, kb, kb, kb, sw);      // T_i is upper triangular (lower zero)
            if (c) {
                // T12 = -T_prev (V_prev^H V_i) T_i over the rows V_i spans
                Scratch S1((size_t)c * kb * sizeof(T), sw), S2((size_t)c * kb * sizeof(T), sw);
                gemm_k<T>(ct, 'N', c, kb, mi, T(1), vg + off, m, Vi, mi, T(0), S1.as<T>(), c, sw);
                gemm_k<T>('N', 'N', c, kb, c, T(1), tg, kt, S1.as<T>(), c, T(0), S2.as<T>(), c, sw);
                gemm_k<T>('N', 'N', c, kb, kb, T(-1), S2.as<T>(), c, Ti, kb, T(0), tg + c * kt, kt, sw);
            }
            c += kb;
        }
        i1 = i0;
    }
}

// Z(r0:, :) -= Vg Tg (Vg^H Z(r0:, :)) per group, on s
template <typename T>
void apply_groups(i64 nc, std::vector<QGroup<T>>& gs, T* Z, i64 ldz, hipStream_t s) {
    const char ct = ctrans<T>();
    if (nc <= 0) return;
    for (auto& g : gs) {
        const i64 kt = g.kt, m = g.m;
        T* vg = g.Vg->template as<T>();
        T* tg = g.Tg->template as<T>();
        Scratch W((size_t)kt * nc * sizeof(T), s), W2((size_t)kt * nc * sizeof(T), s);
        gemm_k<T>(ct, 'N', kt, nc, m, T(1), vg, m, Z + g.r0, ldz, T(0), W.as<T>(), kt, s);
        gemm_k<T>('N', 'N', kt, nc, kt, T(1), tg, kt, W.as<T>(), kt, T(0), W2.as<T>(), kt, s);
        gemm_k<T>('N', 'N', m, nc, kt, T(-1), vg, m, W2.as<T>(), kt, T(1), Z + g.r0, ldz, s);
    }
}

template <typename T>
void unmtr_he2hb(i64 n, i64 nc, std::vector<Panel<T>>& panels, T* Z, i64 ldz, hipStream_t s) {
    const char ct = ctrans<T>();
    const i64 G = unmtr_he2hb_group();
    if (G > 1 && nc > 0) {
        auto gs = he2hb_groups<T>(n, panels, G, s, s, nullptr);
        he2hb_groups_fill<T>(n, panels, G, gs, s);
        apply_groups<T>(nc, gs, Z, ldz, s);
        return;
    }
    for (auto it = panels.rbegin(); it != panels.rend(); ++it) {
        const i64 r0 = it->r0, kk = it->kk, m = n - r0;
        Scratch W((size_t)kk * nc * sizeof(T), s);
        gemm_k<T>(ct, 'N', kk, nc, m, T(1), it->V->template as<T>(), m, Z + r0, ldz, T(0), W.as<T>(), kk, s);
        slate_hip::trmm<K<T>>('L', 'U', 'N', 'N', kk, nc, kv(T(1)), kp(it->T_->template as<T>()), kk,
                              kp(W.as<T>()), kk, s);
        gemm_k<T>('N', 'N', m, nc, kk, T(-1), it->V->template as<T>(), m, W.as<T>(), kk, T(1), Z + r0, ldz, s);
    }
}

// SLATE_AMD_NATIVE_HEEV_DEBUG=1: residual ||M Z - Z diag(w)|| / (||M|| n) of a
// device n x n M (ld ldm) and Z (ld ldz) -- per-stage checks at small n
template <typename T>
void dbg_resid(const char* tag, i64 n, const T* M, i64 ldm, const T* Z, i64 ldz, const std::vector<double>& w,
               hipStream_t s) {
    static const bool on = [] { const char* e = std::getenv("SLATE_AMD_NATIVE_HEEV_DEBUG"); return e && *e == '1'; }();
    if (!on || n > 2048) return;
    NHIP(hipStreamSynchronize(s));
    std::vector<T> m((size_t)n * n), z((size_t)n * n);
    for (i64 j = 0; j < n; ++j) {
        NHIP(hipMemcpy(m.data() + j * n, M + j * ldm, n * sizeof(T), hipMemcpyDeviceToHost));
        NHIP(hipMemcpy(z.data() + j * n, Z + j * ldz, n * sizeof(T), hipMemcpyDeviceToHost));
    }
    double e = 0, an = 0;
    for (i64 j = 0; j < n; ++j)
        for (i64 i = 0; i < n; ++i) {
            T acc = T(0);
            for (i64 l = 0; l < n; ++l) acc += m[i + l * n] * z[l + j * n];
            e += std::norm(acc - z[i + j * n] * (real_t<T>)w[j]);
            an += std::norm(m[i + j * n]);
        }
    std::fprintf(stderr, "heev debug %s: residual %.3e\n", tag, std::sqrt(e / std::max(an, 1e-300)) / (double)n);
}

// the band |i - j| <= b of the dense Af (both triangles) into the skewed
// band layout of the chase (element (i, j) at i + j ldb, ldb = 4b + 8; see
// heev_grid): one block per column, a thread per diagonal offset
template <typename T>
__global__ void band_from_dense_kernel(i64 n, int b, const T* __restrict__ A, i64 lda, T* __restrict__ B, i64 ldb) {
    const i64 j = blockIdx.x;
    const int dlt = (int)threadIdx.x - b;
    if (j >= n || threadIdx.x > 2 * b) return;
    const i64 i = j + dlt;
    if (i < 0 || i >= n) return;
    B[i + j * ldb] = A[i + j * lda];
}

// ---------------------------------------------------------------- one-GPU heev
// Af: dense Hermitian n x n (ld n, both triangles) on this device; w: the
// eigenvalues; Z (n x n, ld n) the eigenvectors when wantz
template <typename T>
void heev_1gpu(i64 n, T* Af, std::vector<double>& w, T* Z, bool wantz, hipStream_t s) {
    using R = real_t<T>;
    const i64 b = std::max<i64>(1, std::min<i64>(64, n - 1));
    std::vector<Panel<T>> panels;
    const bool dbg = [] { const char* e = std::getenv("SLATE_AMD_NATIVE_HEEV_DEBUG"); return e && *e == '1'; }();
    std::unique_ptr<Scratch> A0, B0;
    if (dbg) {
        A0 = std::make_unique<Scratch>((size_t)n * n * sizeof(T), s);
        copy2d(A0->as<T>(), n, Af, n, n, n, s);
    }
    {
        NTRACE("heev::he2hb", s);
        he2hb<T>(n, b, Af, n, panels, s);
    }
    if (dbg) {
        B0 = std::make_unique<Scratch>((size_t)n * n * sizeof(T), s);
        copy2d(B0->as<T>(), n, Af, n, n, n, s);
    }
    // ---- stage 2 on the GPU: bulge chasing with recorded reflectors
    const i64 nsw = std::max<i64>(n - 1, 0);
    std::vector<i64> nt((size_t)std::max<i64>(nsw, 1), 0), sp((size_t)std::max<i64>(n, 1), 0);
    for (i64 j = 0; j < nsw; ++j) {
        const i64 e0 = std::min(j + b, n - 1), k0 = e0 - j;
        nt[j] = k0 <= 1 ? 0 : 1 + (n - 1 - e0 + b - 1) / b;
    }
    for (i64 j = 1; j < n; ++j) sp[j] = sp[j - 1] + nt[j - 1];
    const i64 total = nsw ? sp[n - 1] + nt[nsw - 1] : 0;
    // leading dimension off powers of two (the chase touches ~3b columns of
    // one row band: a 2^k stride would put them on one channel)
    // skewed band layout (default; SLATE_AMD_NATIVE_HB2ST_SKEW=0: the dense
    // n x n copy): the chase touches |i - j| < 2b only, so the band of
    // (4b + 9) n words replaces the n^2 working copy and keeps a task's
    // window contiguous
    static const bool skew = [] { const char* e = std::getenv("SLATE_AMD_NATIVE_HB2ST_SKEW"); return !(e && e[0] == '0'); }() && !dbg;
    const i64 ldp = skew ? 4 * b + 8 : (n + 7) / 8 * 8 + 72;
    const i64 extent = skew ? (n - 1) * (ldp + 1) + 1 : ldp * std::max<i64>(n, 1);
    // the band |i - j| <= b only (models/eig.py _band_only): two masked copies
    Scratch Bh((size_t)(extent + 16) * sizeof(T), s);
    if (skew) {
        dzero(Bh.p, (size_t)(extent + 16) * sizeof(T), s);
        if (n > 0) {
            hipLaunchKernelGGL(band_from_dense_kernel<K<T>>, dim3((unsigned)n), dim3((unsigned)(2 * b + 1)), 0, s, n,
                               (int)b, kp(Af), n, kp(Bh.as<T>()), ldp);
            NHIP(hipGetLastError());
        }
    } else {
        slate_hip::TriMask up_, lo_;
        up_.mode = 2;
        up_.diag_off = b;                       // i <= j + b
        lo_.mode = 1;
        lo_.diag_off = b;                       // i + b >= j
        slate_hip::gecopy_mask<K<T>>(up_, n, n, kp(Af), n, kp(Bh.as<T>()), ldp, false, s);
        slate_hip::gecopy_mask<K<T>>(lo_, n, n, kp(Bh.as<T>()), ldp, kp(Bh.as<T>()), ldp, false, s);
    }
    if (dbg) {
        Scratch Bb((size_t)n * n * sizeof(T), s);
        copy2d(Bb.as<T>(), n, Bh.as<T>(), ldp, n, n, s);
        std::vector<T> h1((size_t)n * n), h2((size_t)n * n);
        NHIP(hipStreamSynchronize(s));
        NHIP(hipMemcpy(h1.data(), Bb.p, h1.size() * sizeof(T), hipMemcpyDeviceToHost));
        NHIP(hipMemcpy(h2.data(), B0->p, h2.size() * sizeof(T), hipMemcpyDeviceToHost));
        double dd = 0, nn = 0;
        for (size_t i = 0; i < h1.size(); ++i) { dd += std::norm(h1[i] - h2[i]); nn += std::norm(h2[i]); }
        std::fprintf(stderr, "heev debug: outside-band part of the stage-1 result %.3e (relative)\n",
                     std::sqrt(dd / std::max(nn, 1e-300)));
    }
    Scratch V((size_t)std::max<i64>(total, 1) * b * sizeof(T), s), tau((size_t)std::max<i64>(total, 1) * sizeof(T), s);
    Scratch row((size_t)std::max<i64>(total, 1) * sizeof(i64), s), len((size_t)std::max<i64>(total, 1) * sizeof(i64), s);
    dzero(V.p, (size_t)std::max<i64>(total, 1) * b * sizeof(T), s);
    dzero(tau.p, (size_t)std::max<i64>(total, 1) * sizeof(T), s);
    std::vector<std::unique_ptr<Scratch>> keep;
    Scratch* ntd = upload_vec(keep, nt, s);
    Scratch* spd = upload_vec(keep, sp, s);
    // side stream: the Q1 group merges run during the chase (which fills
    // ~100 of the 256 CUs) and the Q2 T factors during the D & C
    // (SLATE_AMD_NATIVE_HEEV_OVERLAP=0: everything on s)
    static const bool ovl_env = [] { const char* e = std::getenv("SLATE_AMD_NATIVE_HEEV_OVERLAP"); return !(e && e[0] == '0'); }();
    hipStream_t side = rt().panel;
    const i64 G1 = unmtr_he2hb_group();
    const bool overlap = ovl_env && wantz && !dbg && G1 > 1 && side != nullptr && side != s;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    if (overlap)
        for (auto& e : ev) NHIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    struct EvGuard {
        hipEvent_t* e;
        ~EvGuard() { for (int i = 0; i < 3; ++i) if (e[i]) (void)hipEventDestroy(e[i]); }
    } ev_guard{ev};
    std::vector<QGroup<T>> q1g;
    if (overlap) q1g = he2hb_groups<T>(n, panels, G1, s, side, ev[0]);
    if (nsw > 0 && total > 0) {
        Scratch work((size_t)(nsw + 2) * sizeof(int), s);
        dzero(work.p, (size_t)(nsw + 2) * sizeof(int), s);
        hipDeviceProp_t pr;
        NHIP(hipGetDeviceProperties(&pr, rt().device));
        const i64 nt0 = nt[0] ? nt[0] : 1, lag = 2;
        int nwg = (int)std::min<i64>({std::max<i64>(nsw, 1), (i64)pr.multiProcessorCount,
                                      std::max<i64>(8, std::min(nt0 / lag + 8, nt0 / 3 + 15))});
        // diagnostics: SLATE_AMD_HB2ST_NWG overrides the chase's workgroup count
        // (clamped to [1, min(sweeps, CUs)]: every workgroup must be resident)
        if (const char* e = std::getenv("SLATE_AMD_HB2ST_NWG"); e && std::atoi(e) > 0)
            nwg = (int)std::min<i64>({(i64)std::atoi(e), std::max<i64>(nsw, 1), (i64)pr.multiProcessorCount});
        NTRACE("heev::hb2st", s);
        slate_hip::hb2st_device<K<T>>(n, (int)b, kp(Bh.as<T>()), ldp, kp(V.as<T>()), kp(tau.as<T>()), row.as<i64>(),
                                      len.as<i64>(), spd->as<i64>(), ntd->as<i64>(), work.as<int>(), nsw, nwg, s,
                                      nullptr, extent);
    }
    if (overlap) he2hb_groups_fill<T>(n, panels, G1, q1g, side);
    // ---- (d, e) and the phases that make a complex tridiagonal real
    // the diagonal / sub-diagonal = 1 x n blocks with stride ldp + 1
    Scratch dsub((size_t)2 * std::max<i64>(n, 1) * sizeof(T), s);
    copy2d(dsub.as<T>(), 1, Bh.as<T>(), ldp + 1, 1, n, s);
    if (n > 1) copy2d(dsub.as<T>() + n, 1, Bh.as<T>() + 1, ldp + 1, 1, n - 1, s);
    std::vector<T> ds = download_vec<T>(dsub.p, (size_t)(2 * n), s);
    std::vector<T> diag(ds.begin(), ds.begin() + n), sub(ds.begin() + n, ds.end());
    std::vector<double> d((size_t)n), e((size_t)std::max<i64>(n - 1, 0));
    std::vector<T> ph((size_t)n, T(1));
    for (i64 i = 0; i < n; ++i) d[i] = (double)std::real(diag[i]);
    for (i64 i = 0; i + 1 < n; ++i) {
        if constexpr (is_cplx<T>()) {
            const R a = std::abs(sub[i]);
            const T u = a > R(0) ? sub[i] / a : T(1);
            ph[i + 1] = ph[i] * u;
            e[i] = (double)a;
        } else {
            e[i] = (double)sub[i];
        }
    }
    if (const char* dump = std::getenv("SLATE_AMD_NATIVE_HEEV_DUMP"); dump && *dump) {
        std::FILE* f = std::fopen((std::string(dump) + "/de1.bin").c_str(), "wb");
        if (f) {
            std::fwrite(d.data(), sizeof(double), d.size(), f);
            std::fwrite(e.data(), sizeof(double), e.size(), f);
            std::fclose(f);
        }
    }
    if (!wantz) {
        std::vector<double> ee(e);
        ee.resize((size_t)n, 0.0);
        if (slate_tridiag::steqr_impl<double>(n, d.data(), ee.data(), nullptr, 1, 0))
            throw Error("native heev: the tridiagonal QL iteration did not converge");
        w = d;
        return;
    }
    // ---- tridiagonal eigenvectors (D & C), then Z = Q1 Q2 Phase Qt
    // fp64, b = 64: groups of b reflectors (sweep block J, task t) as block
    // reflectors I - V T V^H on MFMA (eig.hip unmtr_hb2st_mfma, the Python
    // path's form; the register-window kernel below is the other
    // precisions' path).  Their T factors are built first -- on the side
    // stream, during the D & C, when overlapping
    std::vector<i64> gJ, gt, gptr(1, 0);
    std::unique_ptr<Scratch> Tg;
    Scratch *gJd = nullptr, *gtd = nullptr, *gpd = nullptr;
    const bool mfma_q2 = std::is_same<T, double>::value && b == 64 && nsw > 0 && total > 0;
    if (mfma_q2) {
        for (i64 J = 0; J * b < nsw; ++J) {
            const i64 TJ = nt[(size_t)(J * b)];
            for (i64 t = 0; t < TJ; ++t) { gJ.push_back(J); gt.push_back(t); }
            gptr.push_back(gptr.back() + TJ);
        }
        if (!gJ.empty()) {
            gJd = upload_vec(keep, gJ, s);
            gtd = upload_vec(keep, gt, s);
            gpd = upload_vec(keep, gptr, s);
            Tg = std::make_unique<Scratch>(gJ.size() * 2 * b * b * sizeof(double), s);
            hipStream_t st = s;
            if (overlap) {
                NHIP(hipEventRecord(ev[1], s));
                NHIP(hipStreamWaitEvent(side, ev[1], 0));
                st = side;
            }
            if constexpr (std::is_same<T, double>::value)
                slate_hip::unmtr_hb2st_mfma(n, n, nullptr, n, V.as<double>(), b, tau.as<double>(), spd->as<i64>(),
                                            ntd->as<i64>(), gJd->as<i64>(), gtd->as<i64>(), gpd->as<i64>(),
                                            (i64)gJ.size(), Tg->as<double>(), nsw, st, 1);
        }
    }
    if (overlap) NHIP(hipEventRecord(ev[2], side));
    Scratch Qt((size_t)n * n * sizeof(double), s);
    {
        NTRACE("heev::stedc", s);
        stedc_device(n, d, e, w, Qt.as<double>(), n, s);
    }
    Scratch* phd = is_cplx<T>() ? upload_vec(keep, ph, s) : nullptr;
    if (dbg) {
        // the tridiagonal itself as a dense matrix
        std::vector<double> td((size_t)n * n, 0.0);
        for (i64 i = 0; i < n; ++i) td[i + i * n] = d[i];
        for (i64 i = 0; i + 1 < n; ++i) td[i + 1 + i * n] = td[i + (i + 1) * n] = e[i];
        Scratch Td((size_t)n * n * sizeof(double), s);
        upload(Td.p, td.data(), td.size() * sizeof(double), s);
        dbg_resid<double>("tridiagonal D&C", n, Td.as<double>(), n, Qt.as<double>(), n, w, s);
    }
    NTRACE("heev::back_transform", s);
    real_to_phase<T>(n, n, Qt.as<double>(), n, phd ? kp(phd->as<T>()) : nullptr, kp(Z), n, s);
    // the side stream's Q1 merges and Q2 T factors are done before the
    // applies
    if (overlap) NHIP(hipStreamWaitEvent(s, ev[2], 0));
    bool q2_done = false;
    if constexpr (std::is_same<T, double>::value) {
        if (mfma_q2) {
            q2_done = gJ.empty() ||
                      slate_hip::unmtr_hb2st_mfma(n, n, Z, n, V.as<double>(), b, tau.as<double>(), spd->as<i64>(),
                                                  ntd->as<i64>(), gJd->as<i64>(), gtd->as<i64>(), gpd->as<i64>(),
                                                  (i64)gJ.size(), Tg->as<double>(), nsw, s, 2);
        }
    }
    if (nsw > 0 && total > 0 && !q2_done) {
        if (!slate_hip::unmtr_hb2st_blocked<K<T>>(n, n, kp(Z), n, kp(V.as<T>()), b, kp(tau.as<T>()), spd->as<i64>(),
                                                  ntd->as<i64>(), nsw, false, s)) {
            for (i64 j = n - 1; j >= 0; --j) {
                const i64 first = sp[j], last = j + 1 < n ? sp[j + 1] : total;
                if (last > first)
                    slate_hip::apply_refl_batch<K<T>>(n, kp(Z), n, kp(V.as<T>()), b, kp(tau.as<T>()), row.as<i64>(),
                                                      len.as<i64>(), first, last - first, false, s);
            }
        }
    }
    if (dbg) dbg_resid<T>("band (after unmtr_hb2st)", n, B0->as<T>(), n, Z, n, w, s);
    if (overlap) apply_groups<T>(n, q1g, Z, n, s);
    else unmtr_he2hb<T>(n, n, panels, Z, n, s);
    if (dbg) dbg_resid<T>("dense (after unmtr_he2hb)", n, A0->as<T>(), n, Z, n, w, s);
    NHIP(hipStreamSynchronize(s));
}

// ---------------------------------------------------------------- gather / scatter
// every rank's local block -> rank 0's dense n x n (ld n) device copy
template <typename T>
void gather_root(const Storage& S, T* D, hipStream_t s) {
    Runtime& R = rt();
    const int P = S.p * S.q;
    const i64 nb = S.nb;
    auto place = [&](const T* blk, i64 ldb, int pr, int pc) {
        const i64 ml = numroc(S.m, nb, pr, S.p), nl = numroc(S.n, nb, pc, S.q);
        for (i64 lj = 0; lj < nl; lj += nb)
            for (i64 li = 0; li < ml; li += nb) {
                const i64 gi = l2g(li, nb, S.p, pr), gj = l2g(lj, nb, S.q, pc);
                copy2d(D + gi + gj * S.m, S.m, blk + li + lj * ldb, ldb, std::min(nb, ml - li), std::min(nb, nl - lj),
                       s);
            }
    };
    if (P == 1) {
        place(static_cast<const T*>(S.buf), S.lld, 0, 0);
        return;
    }
    std::vector<std::unique_ptr<Scratch>> bufs;
    std::vector<P2P> ops;
    std::vector<std::tuple<int, int, int, Scratch*>> got;
    if (R.rank == 0) {
        place(static_cast<const T*>(S.buf), S.lld, S.pr, S.pc);
        for (int r = 1; r < P; ++r) {
            const int pr = r % S.p, pc = r / S.p;
            const i64 ml = numroc(S.m, nb, pr, S.p), nl = numroc(S.n, nb, pc, S.q);
            if (!ml || !nl) continue;
            bufs.push_back(std::make_unique<Scratch>((size_t)ml * nl * sizeof(T), s));
            ops.push_back({false, r, bufs.back()->p, (size_t)ml * nl * sizeof(T)});
            got.emplace_back(r, pr, pc, bufs.back().get());
        }
    } else if (S.mloc && S.nloc) {
        bufs.push_back(std::make_unique<Scratch>((size_t)S.mloc * S.nloc * sizeof(T), s));
        copy2d(bufs.back()->as<T>(), S.mloc, static_cast<const T*>(S.buf), S.lld, S.mloc, S.nloc, s);
        ops.push_back({true, 0, bufs.back()->p, (size_t)S.mloc * S.nloc * sizeof(T)});
    }
    if (!ops.empty()) world_comm()->exchange(ops, s);
    for (auto& g : got) {
        const int pr = std::get<1>(g);
        place(std::get<3>(g)->template as<T>(), numroc(S.m, nb, pr, S.p), pr, std::get<2>(g));
    }
    NHIP(hipStreamSynchronize(s));
}

// rank 0's dense n x n (ld n) device matrix -> every rank's local block of Z
template <typename T>
void scatter_root(const T* D, Storage& S, hipStream_t s) {
    Runtime& R = rt();
    const int P = S.p * S.q;
    const i64 nb = S.nb;
    auto take = [&](T* blk, i64 ldb, int pr, int pc) {
        const i64 ml = numroc(S.m, nb, pr, S.p), nl = numroc(S.n, nb, pc, S.q);
        for (i64 lj = 0; lj < nl; lj += nb)
            for (i64 li = 0; li < ml; li += nb) {
                const i64 gi = l2g(li, nb, S.p, pr), gj = l2g(lj, nb, S.q, pc);
                copy2d(blk + li + lj * ldb, ldb, D + gi + gj * S.m, S.m, std::min(nb, ml - li), std::min(nb, nl - lj),
                       s);
            }
    };
    if (P == 1) {
        take(static_cast<T*>(S.buf), S.lld, 0, 0);
        NHIP(hipStreamSynchronize(s));
        return;
    }
    std::vector<std::unique_ptr<Scratch>> bufs;
    std::vector<P2P> ops;
    Scratch* mine = nullptr;
    if (R.rank == 0) {
        take(static_cast<T*>(S.buf), S.lld, S.pr, S.pc);
        for (int r = 1; r < P; ++r) {
            const int pr = r % S.p, pc = r / S.p;
            const i64 ml = numroc(S.m, nb, pr, S.p), nl = numroc(S.n, nb, pc, S.q);
            if (!ml || !nl) continue;
            bufs.push_back(std::make_unique<Scratch>((size_t)ml * nl * sizeof(T), s));
            take(bufs.back()->as<T>(), ml, pr, pc);
            ops.push_back({true, r, bufs.back()->p, (size_t)ml * nl * sizeof(T)});
        }
    } else if (S.mloc && S.nloc) {
        bufs.push_back(std::make_unique<Scratch>((size_t)S.mloc * S.nloc * sizeof(T), s));
        mine = bufs.back().get();
        ops.push_back({false, 0, mine->p, (size_t)S.mloc * S.nloc * sizeof(T)});
    }
    if (!ops.empty()) world_comm()->exchange(ops, s);
    if (mine) copy2d(static_cast<T*>(S.buf), S.lld, mine->as<T>(), S.mloc, S.mloc, S.nloc, s);
    NHIP(hipStreamSynchronize(s));
}

// the full Hermitian (both triangles, real diagonal) from its uplo triangle
template <typename T>
void symmetrize(i64 n, T* D, Uplo uplo, hipStream_t s) {
    if (n <= 0) return;
    Scratch Tt((size_t)n * n * sizeof(T), s);
    slate_hip::TriMask keep, other;
    keep.mode = uplo == Uplo::Lower ? 1 : 2;
    other.mode = uplo == Uplo::Lower ? 2 : 1;
    other.diag_off = -1;                    // the strict opposite triangle
    slate_hip::gecopy_mask<K<T>>(keep, n, n, kp(D), n, kp(D), n, true, s);           // stored triangle, real diagonal
    slate_hip::gecopy<K<T>, K<T>>('G', ctrans<T>(), n, n, kp(D), n, kp(Tt.as<T>()), n, s);
    slate_hip::gecopy_mask_merge<K<T>>(other, n, n, kp(Tt.as<T>()), n, kp(D), n, s);
}

// ================================================================ heev on a p x q grid
// No rank ever holds an n x n matrix (models/eig_dist.py is the Python twin;
// reference src/heev.cc:132-205, src/he2hb.cc:26-677, he2hbGather of
// HermitianBandMatrix.hh:310, src/unmtr_hb2st.cc, src/unmtr_he2hb.cc):
//   * F = A with both triangles on A's grid with tile b = 64 (redistribute);
//   * he2hb_grid: per panel the tile column is all-gathered inside its
//     process column and QR-factored there (redundantly, deterministic
//     kernels), the factored rows written back (R + reflectors, the SLATE
//     layout), V and T broadcast along the process rows; Y = A22 V T is one
//     local GEMM summed over the process row, M = (V T)^H Y summed over the
//     process column, W = Y - V M / 2 assembled by one column all-reduce,
//     and A22 -= [V W] [W V]^H is one local GEMM of inner size 2b;
//   * the band (O(n b) words) is summed to every rank; rank 0 chases it on
//     the GPU in a SKEWED band layout (element (i, j) at i + j lda with
//     lda = 4b + 8: the chase only touches |i - j| < 2b, so the dense-window
//     kernel runs on (4b + 9) n words instead of n^2);
//   * divide & conquer with the eigenvector rows distributed (stedc_rows);
//   * Q2 (the chase's reflectors) on a 1 x P column-cyclic Z, the reflectors
//     streamed from rank 0 in chunks of sweep blocks (never all n^2 / 2 words
//     at once); Q1 on F's grid, the panel reflectors read back from F and
//     broadcast along the process rows; Z onto the caller's layout.
// Every layout change is one redistribute() (separable owner blocks, one
// batched point-to-point exchange).
template <typename T>
struct GPanel { i64 k, r0, kk; std::unique_ptr<Scratch> T_; };

template <typename T>
__global__ void band_from_stack_kernel(i64 n, int b, const T* __restrict__ st, i64 lds, T* __restrict__ A, i64 lda) {
    // one thread per (i - j, j) with |i - j| <= b; the stack holds, per tile
    // column k (columns k b ..), the diagonal tile's lower triangle in rows
    // [0, b) and the sub-diagonal R block's upper triangle in rows [b, 2b)
    const i64 j = blockIdx.x;
    const int dlt = (int)threadIdx.x - b;              // i - j
    if (j >= n || threadIdx.x > 2 * b) return;
    const i64 i = j + dlt;
    if (i < 0 || i >= n) return;
    const i64 r = i > j ? i : j, c = i > j ? j : i;    // the lower-triangle element
    const i64 c0 = (c / b) * b;
    const T v = (r < c0 + b) ? st[(r - c0) + c * lds] : st[b + (r - c0 - b) + c * lds];
    T out = v;
    if (i == j) {
        if constexpr (slate_hip::scalar_traits<T>::is_complex) out.im = 0;
    } else if (i < j) {
        out = slate_hip::s_conj(v);
    }
    A[i + j * lda] = out;
}

template <typename T>
void he2hb_grid(Storage& F, std::vector<GPanel<T>>& pans, hipStream_t s) {
    GridComms* gc = F.gc;
    const int p = F.p, q = F.q, pr = F.pr, pc = F.pc;
    const i64 nb = F.nb, n = F.n, mloc = F.mloc, nloc = F.nloc, lld = F.lld;
    const i64 nt = (n + nb - 1) / nb;
    T* buf = static_cast<T*>(F.buf);
    const char ct = ctrans<T>();
    const size_t es = sizeof(T);
    std::vector<std::unique_ptr<Scratch>> keep;
    for (i64 k = 0; k + 1 < nt; ++k) {
        keep.clear();
        const i64 r0 = (k + 1) * nb, kb = std::min(nb, n - k * nb), m2 = n - r0, kk = std::min(m2, kb);
        const int ck = (int)(k % q);
        const i64 lr0 = std::min(tiles_before(k + 1, p, pr) * nb, mloc), nmine = mloc - lr0;
        const i64 lc_k = tiles_before(k, q, pc) * nb;
        const i64 lc1 = std::min(tiles_before(k + 1, q, pc) * nb, nloc), ncl = nloc - lc1;
        std::vector<i64> rowidx((size_t)nmine), colidx((size_t)ncl);
        for (i64 r = 0; r < nmine; ++r) rowidx[r] = l2g(lr0 + r, nb, p, pr) - r0;
        for (i64 c = 0; c < ncl; ++c) colidx[c] = l2g(lc1 + c, nb, q, pc) - r0;
        i64* rid = upload_vec(keep, rowidx, s)->template as<i64>();
        i64* cid = upload_vec(keep, colidx, s)->template as<i64>();
        Scratch VT((size_t)(m2 * kk + kk * kk) * es, s);
        T* Vf = VT.as<T>();
        T* Tk = Vf + m2 * kk;
        if (pc == ck) {
            // the panel rows of every process row, padded to the longest
            std::vector<i64> cnt((size_t)p);
            i64 maxc = 1;
            for (int r = 0; r < p; ++r) {
                const i64 ml = numroc(n, nb, r, p);
                cnt[r] = ml - std::min(tiles_before(k + 1, p, r) * nb, ml);
                maxc = std::max(maxc, cnt[r]);
            }
            Scratch snd((size_t)maxc * kb * es, s), rcv((size_t)p * maxc * kb * es, s);
            copy2d(snd.as<T>(), maxc, buf + lr0 + lc_k * lld, lld, nmine, kb, s);
            if (p > 1) gc->col->allgather(snd.p, rcv.p, (size_t)maxc * kb * es, s);
            else dcopy(rcv.p, snd.p, (size_t)maxc * kb * es, s);
            Scratch Pf((size_t)m2 * kb * es, s), tau((size_t)kk * es, s);
            for (int r = 0; r < p; ++r) {
                if (!cnt[r]) continue;
                const i64 l0 = std::min(tiles_before(k + 1, p, r) * nb, numroc(n, nb, r, p));
                std::vector<i64> g((size_t)cnt[r]);
                for (i64 i = 0; i < cnt[r]; ++i) g[i] = l2g(l0 + i, nb, p, r) - r0;
                slate_hip::permute_rows_scatter<K<T>>(cnt[r], kb, kp(rcv.as<T>() + (i64)r * maxc * kb), maxc,
                                                      kp(Pf.as<T>()), m2, upload_vec(keep, g, s)->template as<i64>(),
                                                      s);
            }
            dzero(tau.p, (size_t)kk * es, s);
            slate_hip::geqrf_panel_ws<K<T>>(m2, kb, kp(Pf.as<T>()), m2, kp(tau.as<T>()), kp(Tk), kk, kp(Vf), m2,
                                            rt().qr_work, s);
            // R and the reflectors back into this rank's rows of the panel
            slate_hip::permute_rows_gather<K<T>>(nmine, kb, kp(Pf.as<T>()), m2, kp(buf + lr0 + lc_k * lld), lld, rid,
                                                 s);
        }
        if (q > 1) gc->row->bcast(VT.p, (size_t)(m2 * kk + kk * kk) * es, ck, s);
        GPanel<T> pn{k, r0, kk, std::make_unique<Scratch>((size_t)kk * kk * es, s)};
        copy2d(pn.T_->template as<T>(), kk, Tk, kk, kk, kk, s);
        pans.push_back(std::move(pn));
        // X = V T (every rank, m2 x kk)
        Scratch X((size_t)m2 * kk * es, s);
        copy2d(X.as<T>(), m2, Vf, m2, m2, kk, s);
        slate_hip::trmm<K<T>>('R', 'U', 'N', 'N', m2, kk, kv(T(1)), kp(Tk), kk, kp(X.as<T>()), m2, s);
        // Y = A22 X(my columns), summed over the process row
        const i64 ldy = std::max<i64>(nmine, 1);
        Scratch VW((size_t)ldy * 2 * kk * es, s);       // [V_mine | W_mine]
        T* Vl = VW.as<T>();
        T* Y = Vl + ldy * kk;
        if (nmine) {
            if (ncl) {
                Scratch Xc((size_t)ncl * kk * es, s);
                slate_hip::permute_rows_gather<K<T>>(ncl, kk, kp(X.as<T>()), m2, kp(Xc.as<T>()), ncl, cid, s);
                gemm_k<T>('N', 'N', nmine, kk, ncl, T(1), buf + lr0 + lc1 * lld, lld, Xc.as<T>(), ncl, T(0), Y, ldy, s);
            } else {
                slate_hip::geset<K<T>>('G', nmine, kk, kv(T(0)), kv(T(0)), kp(Y), ldy, s);
            }
            if (q > 1) gc->row->allreduce(Y, (size_t)(ldy * kk), dt_of<T>::v, 's', s);
        }
        // M = X(my rows)^H Y, summed over the process column
        Scratch M((size_t)kk * kk * es, s);
        if (nmine) {
            Scratch Xl((size_t)nmine * kk * es, s);
            slate_hip::permute_rows_gather<K<T>>(nmine, kk, kp(X.as<T>()), m2, kp(Xl.as<T>()), nmine, rid, s);
            gemm_k<T>(ct, 'N', kk, kk, nmine, T(1), Xl.as<T>(), nmine, Y, ldy, T(0), M.as<T>(), kk, s);
            slate_hip::permute_rows_gather<K<T>>(nmine, kk, kp(Vf), m2, kp(Vl), ldy, rid, s);
        } else {
            slate_hip::geset<K<T>>('G', kk, kk, kv(T(0)), kv(T(0)), kp(M.as<T>()), kk, s);
        }
        if (p > 1) gc->col->allreduce(M.p, (size_t)(kk * kk), dt_of<T>::v, 's', s);
        // W = Y - V M / 2, then the full W (m2 x kk) by one column all-reduce
        if (nmine) gemm_k<T>('N', 'N', nmine, kk, kk, T(-0.5), Vl, ldy, M.as<T>(), kk, T(1), Y, ldy, s);
        Scratch Wf((size_t)m2 * kk * es, s);
        dzero(Wf.p, (size_t)m2 * kk * es, s);
        if (nmine) slate_hip::permute_rows_scatter<K<T>>(nmine, kk, kp(Y), ldy, kp(Wf.as<T>()), m2, rid, s);
        if (p > 1) gc->col->allreduce(Wf.p, (size_t)(m2 * kk), dt_of<T>::v, 's', s);
        // A22 -= [V W] [W V]^H over my trailing block (one GEMM, inner 2 kk)
        if (nmine && ncl) {
            Scratch WV((size_t)ncl * 2 * kk * es, s);
            slate_hip::permute_rows_gather<K<T>>(ncl, kk, kp(Wf.as<T>()), m2, kp(WV.as<T>()), ncl, cid, s);
            slate_hip::permute_rows_gather<K<T>>(ncl, kk, kp(Vf), m2, kp(WV.as<T>() + ncl * kk), ncl, cid, s);
            gemm_k<T>('N', ct, nmine, ncl, 2 * kk, T(-1), Vl, ldy, WV.as<T>(), ncl, T(1), buf + lr0 + lc1 * lld, lld, s);
        }
        NHIP(hipStreamSynchronize(s));
    }
}

// Z := Q1 Z on F's grid (Z shares F's layout); panels last to first, G
// consecutive panels merged into one block reflector (as the one-GPU
// unmtr_he2hb): Vg = this rank's rows of the group's reflectors (each
// panel's rows broadcast along the process row from its owner column),
// Tg from the forward larft merge with V_prev^H V_i summed over the process
// column -- one W = Vg^H Z all-reduce per group instead of per panel.
template <typename T>
void unmtr_he2hb_grid(const Storage& F, std::vector<GPanel<T>>& pans, Storage& Zs, hipStream_t s) {
    GridComms* gc = F.gc;
    const int p = F.p, q = F.q, pr = F.pr, pc = F.pc;
    const i64 nb = F.nb, mloc = F.mloc, lld = F.lld, nz = Zs.nloc, ldz = Zs.lld;
    const T* fb = static_cast<const T*>(F.buf);
    T* Z = static_cast<T*>(Zs.buf);
    const char ct = ctrans<T>();
    const size_t es = sizeof(T);
    static const i64 G = [] { const char* e = std::getenv("SLATE_AMD_UNMTR_HE2HB_GROUP"); return e ? std::max(1, std::atoi(e)) : 4; }();
    // this rank's rows of panel i's reflectors (nmine_i x kk_i, ld max(nmine_i, 1)), every rank of the row
    auto panel_rows = [&](const GPanel<T>& pn, i64& lr0, i64& nmine) {
        const i64 k = pn.k, kk = pn.kk;
        const int ck = (int)(k % q);
        lr0 = std::min(tiles_before(k + 1, p, pr) * nb, mloc);
        nmine = mloc - lr0;
        const i64 lc_k = tiles_before(k, q, pc) * nb;
        auto V = std::make_unique<Scratch>((size_t)std::max<i64>(nmine, 1) * kk * es, s);
        if (nmine) {
            if (pc == ck) {
                if (pr == (int)((k + 1) % p))
                    slate_hip::v_explicit<K<T>>(nmine, kk, kp(fb + lr0 + lc_k * lld), lld, kp(V->template as<T>()),
                                                nmine, s);
                else
                    copy2d(V->template as<T>(), nmine, fb + lr0 + lc_k * lld, lld, nmine, kk, s);
            }
            if (q > 1) gc->row->bcast(V->p, (size_t)nmine * kk * es, ck, s);
        }
        return V;
    };
    if (G > 1) {
        i64 i1 = (i64)pans.size();
        while (i1 > 0) {
            const i64 i0 = std::max<i64>(0, i1 - G);
            i64 kt = 0;
            for (i64 i = i0; i < i1; ++i) kt += pans[i].kk;
            const i64 lrg = std::min(tiles_before(pans[i0].k + 1, p, pr) * nb, mloc), mg = mloc - lrg;
            const i64 ldv = std::max<i64>(mg, 1);
            Scratch Vg((size_t)ldv * kt * es, s), Tg((size_t)kt * kt * es, s);
            dzero(Vg.p, (size_t)ldv * kt * es, s);
            dzero(Tg.p, (size_t)kt * kt * es, s);
            T* vg = Vg.as<T>();
            T* tg = Tg.as<T>();
            i64 c = 0;
            for (i64 i = i0; i < i1; ++i) {
                i64 lr0 = 0, nmine = 0;
                const auto V = panel_rows(pans[i], lr0, nmine);
                const i64 kb = pans[i].kk, off = lr0 - lrg;
                if (nmine) copy2d(vg + off + c * ldv, ldv, V->template as<T>(), nmine, nmine, kb, s);
                copy2d(tg + c + c * kt, kt, pans[i].T_->template as<T>(), kb, kb, kb, s);
                if (c) {
                    // T12 = -T_prev (V_prev^H V_i) T_i, V_prev^H V_i summed over the process column
                    Scratch S1((size_t)c * kb * es, s), S2((size_t)c * kb * es, s);
                    if (nmine)
                        gemm_k<T>(ct, 'N', c, kb, nmine, T(1), vg + off, ldv, V->template as<T>(), nmine, T(0),
                                  S1.as<T>(), c, s);
                    else
                        slate_hip::geset<K<T>>('G', c, kb, kv(T(0)), kv(T(0)), kp(S1.as<T>()), c, s);
                    if (p > 1) gc->col->allreduce(S1.p, (size_t)(c * kb), dt_of<T>::v, 's', s);
                    gemm_k<T>('N', 'N', c, kb, c, T(1), tg, kt, S1.as<T>(), c, T(0), S2.as<T>(), c, s);
                    gemm_k<T>('N', 'N', c, kb, kb, T(-1), S2.as<T>(), c, pans[i].T_->template as<T>(), kb, T(0),
                              tg + c * kt, kt, s);
                }
                c += kb;
                NHIP(hipStreamSynchronize(s));
            }
            if (nz) {
                Scratch W((size_t)kt * nz * es, s), W2((size_t)kt * nz * es, s);
                if (mg) gemm_k<T>(ct, 'N', kt, nz, mg, T(1), vg, ldv, Z + lrg, ldz, T(0), W.as<T>(), kt, s);
                else slate_hip::geset<K<T>>('G', kt, nz, kv(T(0)), kv(T(0)), kp(W.as<T>()), kt, s);
                if (p > 1) gc->col->allreduce(W.p, (size_t)(kt * nz), dt_of<T>::v, 's', s);
                gemm_k<T>('N', 'N', kt, nz, kt, T(1), tg, kt, W.as<T>(), kt, T(0), W2.as<T>(), kt, s);
                if (mg) gemm_k<T>('N', 'N', mg, nz, kt, T(-1), vg, ldv, W2.as<T>(), kt, T(1), Z + lrg, ldz, s);
            }
            NHIP(hipStreamSynchronize(s));
            i1 = i0;
        }
        return;
    }
    for (auto it = pans.rbegin(); it != pans.rend(); ++it) {
        const i64 k = it->k, kk = it->kk;
        const int ck = (int)(k % q);
        const i64 lr0 = std::min(tiles_before(k + 1, p, pr) * nb, mloc), nmine = mloc - lr0;
        const i64 lc_k = tiles_before(k, q, pc) * nb;
        Scratch Vl((size_t)std::max<i64>(nmine, 1) * kk * es, s);
        if (nmine) {
            if (pc == ck) {
                if (pr == (int)((k + 1) % p))
                    slate_hip::v_explicit<K<T>>(nmine, kk, kp(fb + lr0 + lc_k * lld), lld, kp(Vl.as<T>()), nmine, s);
                else
                    copy2d(Vl.as<T>(), nmine, fb + lr0 + lc_k * lld, lld, nmine, kk, s);
            }
            if (q > 1) gc->row->bcast(Vl.p, (size_t)nmine * kk * es, ck, s);
        }
        if (!nz) continue;
        Scratch W((size_t)kk * nz * es, s);
        if (nmine) gemm_k<T>(ct, 'N', kk, nz, nmine, T(1), Vl.as<T>(), nmine, Z + lr0, ldz, T(0), W.as<T>(), kk, s);
        else slate_hip::geset<K<T>>('G', kk, nz, kv(T(0)), kv(T(0)), kp(W.as<T>()), kk, s);
        if (p > 1) gc->col->allreduce(W.p, (size_t)(kk * nz), dt_of<T>::v, 's', s);
        slate_hip::trmm<K<T>>('L', 'U', 'N', 'N', kk, nz, kv(T(1)), kp(it->T_->template as<T>()), kk,
                              kp(W.as<T>()), kk, s);
        if (nmine) gemm_k<T>('N', 'N', nmine, nz, kk, T(-1), Vl.as<T>(), nmine, W.as<T>(), kk, T(1), Z + lr0, ldz, s);
        NHIP(hipStreamSynchronize(s));
    }
}

// peak device memory of the last heev_grid call on this rank (tests)
size_t g_heev_grid_peak = 0;

template <typename T>
int64_t heev_grid(HermitianMatrix<T>& A, std::vector<real_t<T>>& Lambda, Matrix<T>* Z) {
    NTRACE("heev", nullptr);
    using Rl = real_t<T>;
    Runtime& R = rt();
    hipStream_t s = R.main;
    const Storage& SA = *A.storage();
    const i64 n = SA.n, b = 64;
    const int p = SA.p, q = SA.q, P = R.size;
    Comm* world = world_comm();
    size_t free0 = 0, total0 = 0, low = (size_t)-1;
    auto mark = [&] {
        size_t f = 0, t = 0;
        NHIP(hipMemGetInfo(&f, &t));
        low = std::min(low, f);
    };
    NHIP(hipStreamSynchronize(s));
    NHIP(hipMemGetInfo(&free0, &total0));
    // diagnostics: SLATE_AMD_HEEV_GRID_STOP=k returns after stage k (bisection)
    const int stop = [] { const char* e = std::getenv("SLATE_AMD_HEEV_GRID_STOP"); return e ? std::atoi(e) : 0; }();
    auto stop_at = [&](int k) {
        if (stop != k) return false;
        NHIP(hipStreamSynchronize(s));
        Lambda.assign((size_t)n, 0);
        return true;
    };
    // ---- F: both triangles, tile b, A's grid
    Matrix<T> F(n, n, b, p, q);
    {
        const Matrix<T> Af = expand_tri<T>(A, A.uplo(), 1);
        redistribute<T>(Af, F);
        mark();
    }
    if (stop_at(1)) return 0;
    std::vector<GPanel<T>> pans;
    {
        NTRACE("heev::he2hb", s);
        he2hb_grid<T>(*F.storage(), pans, s);
    }
    mark();
    if (stop_at(2)) return 0;
    // ---- the band to every rank (O(n b)), stage 2 on rank 0
    const Storage& SF = *F.storage();
    const i64 nt = (n + b - 1) / b;
    Scratch stack((size_t)2 * b * n * sizeof(T), s);
    dzero(stack.p, (size_t)2 * b * n * sizeof(T), s);
    for (i64 k = 0; k < nt; ++k) {
        if ((int)(k % q) != SF.pc) continue;
        const i64 c0 = k * b, kb = std::min(b, n - c0), lc = tiles_before(k, q, SF.pc) * b;
        const T* fb = static_cast<const T*>(SF.buf);
        if ((int)(k % p) == SF.pr)
            copy2d(stack.as<T>() + c0 * 2 * b, 2 * b, fb + tiles_before(k, p, SF.pr) * b + lc * SF.lld, SF.lld, kb, kb, s);
        if (k + 1 < nt && (int)((k + 1) % p) == SF.pr)
            copy2d(stack.as<T>() + b + c0 * 2 * b, 2 * b, fb + tiles_before(k + 1, p, SF.pr) * b + lc * SF.lld, SF.lld,
                   std::min(b, n - (k + 1) * b), kb, s);
    }
    if (P > 1) world->allreduce(stack.p, (size_t)(2 * b * n), dt_of<T>::v, 's', s);
    const i64 nsw = std::max<i64>(n - 1, 0);
    std::vector<i64> ntk((size_t)std::max<i64>(nsw, 1), 0), sp((size_t)std::max<i64>(n, 1), 0);
    for (i64 j = 0; j < nsw; ++j) {
        const i64 e0 = std::min(j + b, n - 1), k0 = e0 - j;
        ntk[j] = k0 <= 1 ? 0 : 1 + (n - 1 - e0 + b - 1) / b;
    }
    for (i64 j = 1; j < n; ++j) sp[j] = sp[j - 1] + ntk[j - 1];
    const i64 total = nsw ? sp[n - 1] + ntk[nsw - 1] : 0;
    std::vector<std::unique_ptr<Scratch>> keep;
    Scratch* ntd = upload_vec(keep, ntk, s);
    Scratch* spd = upload_vec(keep, sp, s);
    const bool cplx = is_cplx<T>();
    // host record broadcast from rank 0: d (n), e (n - 1), phases (2n), error
    std::vector<double> rec((size_t)(n + std::max<i64>(n - 1, 0) + 2 * n + 1), 0.0);
    std::unique_ptr<Scratch> V2, tau2;
    std::string msg;
    if (R.rank == 0) {
        try {
            NTRACE("heev::hb2st", s);
            // element (i, j), |i - j| < 2b, at i + j lda: row i - j of column j
            // of a band of leading dimension lda + 1; the highest address is
            // (n - 1)(lda + 1), so the chase gets that extent (not lda n)
            const i64 lda = 4 * b + 8;
            const i64 extent = (n - 1) * (lda + 1) + 1;
            const size_t words = (size_t)(extent + 16);
            Scratch Bh(words * sizeof(T), s);
            dzero(Bh.p, words * sizeof(T), s);
            T* Ab = Bh.as<T>();
            hipLaunchKernelGGL(band_from_stack_kernel<K<T>>, dim3((unsigned)n), dim3((unsigned)(2 * b + 1)), 0, s,
                               n, (int)b, kp(stack.as<T>()), 2 * b, kp(Ab), lda);
            NHIP(hipGetLastError());
            if (const char* dump = std::getenv("SLATE_AMD_NATIVE_HEEV_DUMP"); dump && *dump) {
                const std::vector<T> hb = download_vec<T>(Bh.p, words, s);
                std::FILE* f = std::fopen((std::string(dump) + "/skew.bin").c_str(), "wb");
                if (f) { std::fwrite(hb.data(), sizeof(T), hb.size(), f); std::fclose(f); }
            }
            V2 = std::make_unique<Scratch>((size_t)std::max<i64>(total, 1) * b * sizeof(T), s);
            tau2 = std::make_unique<Scratch>((size_t)std::max<i64>(total, 1) * sizeof(T), s);
            Scratch row((size_t)std::max<i64>(total, 1) * sizeof(i64), s), len((size_t)std::max<i64>(total, 1) * sizeof(i64), s);
            dzero(V2->p, (size_t)std::max<i64>(total, 1) * b * sizeof(T), s);
            dzero(tau2->p, (size_t)std::max<i64>(total, 1) * sizeof(T), s);
            if (nsw > 0 && total > 0) {
                Scratch work((size_t)(nsw + 2) * sizeof(int), s);
                dzero(work.p, (size_t)(nsw + 2) * sizeof(int), s);
                hipDeviceProp_t prp;
                NHIP(hipGetDeviceProperties(&prp, R.device));
                const i64 nt0 = ntk[0] ? ntk[0] : 1, lag = 2;
                const int nwg = (int)std::min<i64>({std::max<i64>(nsw, 1), (i64)prp.multiProcessorCount,
                                                    std::max<i64>(8, std::min(nt0 / lag + 8, nt0 / 3 + 15))});
                slate_hip::hb2st_device<K<T>>(n, (int)b, kp(Ab), lda, kp(V2->template as<T>()),
                                              kp(tau2->template as<T>()), row.as<i64>(), len.as<i64>(),
                                              spd->as<i64>(), ntd->as<i64>(), work.as<int>(), nsw, nwg, s, nullptr,
                                              extent);
            }
            Scratch dsub((size_t)2 * n * sizeof(T), s);
            copy2d(dsub.as<T>(), 1, Ab, lda + 1, 1, n, s);
            if (n > 1) copy2d(dsub.as<T>() + n, 1, Ab + 1, lda + 1, 1, n - 1, s);
            const std::vector<T> ds = download_vec<T>(dsub.p, (size_t)(2 * n), s);
            std::vector<T> ph((size_t)n, T(1));
            for (i64 i = 0; i < n; ++i) rec[i] = (double)std::real(ds[i]);
            for (i64 i = 0; i + 1 < n; ++i) {
                const T sub = ds[n + i];
                if constexpr (is_cplx<T>()) {
                    const Rl a = std::abs(sub);
                    const T u = a > Rl(0) ? sub / a : T(1);
                    ph[i + 1] = ph[i] * u;
                    rec[n + i] = (double)a;
                } else {
                    rec[n + i] = (double)sub;
                }
            }
            const i64 po = n + std::max<i64>(n - 1, 0);
            for (i64 i = 0; i < n; ++i) {
                rec[po + 2 * i] = (double)std::real(ph[i]);
                rec[po + 2 * i + 1] = (double)std::imag(ph[i]);
            }
            mark();
        } catch (const std::exception& e) {
            rec.back() = 1;
            msg = e.what();
        }
    }
    if (P > 1) {
        Scratch rb(rec.size() * sizeof(double), s);
        if (R.rank == 0) upload(rb.p, rec.data(), rec.size() * sizeof(double), s);
        world->bcast(rb.p, rec.size() * sizeof(double), 0, s);
        rec = download_vec<double>(rb.p, rec.size(), s);
    }
    if (rec.back() != 0) throw Error(R.rank == 0 ? msg : std::string("native heev: stage 2 failed on rank 0"));
    if (const char* dump = std::getenv("SLATE_AMD_NATIVE_HEEV_DUMP"); dump && *dump && R.rank == 0) {
        // diagnostics: the gathered band stack (2b x n) and (d, e), raw binary
        const std::vector<T> hs = download_vec<T>(stack.p, (size_t)(2 * b * n), s);
        std::FILE* f = std::fopen((std::string(dump) + "/stack.bin").c_str(), "wb");
        if (f) { std::fwrite(hs.data(), sizeof(T), hs.size(), f); std::fclose(f); }
        f = std::fopen((std::string(dump) + "/de.bin").c_str(), "wb");
        if (f) { std::fwrite(rec.data(), sizeof(double), (size_t)(2 * n - 1), f); std::fclose(f); }
    }
    std::vector<double> d(rec.begin(), rec.begin() + n), e(rec.begin() + n, rec.begin() + n + std::max<i64>(n - 1, 0));
    std::vector<double> w;
    if (stop_at(3)) return 0;
    if (!Z) {
        std::vector<double> ee(e);
        ee.resize((size_t)n, 0.0);
        if (slate_tridiag::steqr_impl<double>(n, d.data(), ee.data(), nullptr, 1, 0))
            throw Error("native heev: the tridiagonal QL iteration did not converge");
        Lambda.assign(d.begin(), d.end());
        return 0;
    }
    // ---- tridiagonal eigenvectors, rows distributed: rank r rows [r mb, ...)
    const i64 mb = (n + P - 1) / P;
    Matrix<T> Zrow(n, n, mb, P, 1);
    if (stop_at(31)) return 0;
    {
        NTRACE("heev::stedc", s);
        const Storage& SR = *Zrow.storage();
        const i64 r0 = std::min<i64>((i64)R.rank * mb, n), nr = SR.mloc;
        Scratch Qr((size_t)std::max<i64>(nr, 1) * n * sizeof(double), s);
        if (std::getenv("SLATE_AMD_HEEV_GRID_DCFULL")) {
            // diagnostics: the one-process D&C (all rows) on every rank
            Scratch Qf((size_t)n * n * sizeof(double), s);
            stedc_rows(n, d, e, w, Qf.as<double>(), n, 0, n, nullptr, s);
            if (nr) copy2d(Qr.as<double>(), std::max<i64>(nr, 1), Qf.as<double>() + r0, n, nr, n, s);
            NHIP(hipStreamSynchronize(s));
        } else if (const char* dm = std::getenv("SLATE_AMD_HEEV_GRID_DCMODE"); dm && !std::strcmp(dm, "nocomm")) {
            stedc_rows(n, d, e, w, Qr.as<double>(), std::max<i64>(nr, 1), r0, r0 + nr, nullptr, s);
        } else if (dm && !std::strcmp(dm, "fullcomm")) {
            Scratch Qf((size_t)n * n * sizeof(double), s);
            stedc_rows(n, d, e, w, Qf.as<double>(), n, 0, n, world, s);
            NHIP(hipStreamSynchronize(s));
        } else {
            stedc_rows(n, d, e, w, Qr.as<double>(), std::max<i64>(nr, 1), r0, r0 + nr, world, s);
        }
        mark();
        if (stop_at(32)) return 0;
        std::vector<T> ph((size_t)n);
        const i64 po = n + std::max<i64>(n - 1, 0);
        for (i64 i = 0; i < n; ++i) {
            if constexpr (is_cplx<T>()) ph[i] = T((Rl)rec[po + 2 * i], (Rl)rec[po + 2 * i + 1]);
            else ph[i] = T(1);
        }
        Scratch* phd = cplx ? upload_vec(keep, ph, s) : nullptr;
        if (nr) real_to_phase<T>(nr, n, Qr.as<double>(), std::max<i64>(nr, 1), phd ? kp(phd->as<T>() + r0) : nullptr,
                                 kp(static_cast<T*>(SR.buf)), SR.lld, s);
        NHIP(hipStreamSynchronize(s));
    }
    if (stop_at(4)) {
        if (std::getenv("SLATE_AMD_HEEV_GRID_TRIM")) { NHIP(hipDeviceSynchronize()); slate_hip::dev_trim(); }
        return 0;
    }
    // ---- Q2 on a 1 x P column-cyclic Z, reflectors streamed from rank 0
    Matrix<T> Zc(n, n, b, 1, P);
    redistribute<T>(Zrow, Zc);
    Zrow = Matrix<T>();
    {
        NTRACE("heev::unmtr_hb2st", s);
        Storage& SC = *Zc.storage();
        const i64 ncols = SC.nloc;
        const i64 nblk = nsw > 0 ? (nsw - 1) / b + 1 : 0;
        const i64 G = std::max<i64>(1, ncols / 256);          // sweep blocks per chunk (~ <= a quarter of Zc's block)
        for (i64 Jhi = nblk - 1; Jhi >= 0 && total > 0; Jhi -= G) {
            const i64 Jlo = std::max<i64>(0, Jhi - G + 1);
            const i64 s0 = sp[Jlo * b], s1 = (Jhi + 1) * b < nsw ? sp[(Jhi + 1) * b] : total;
            if (s1 <= s0) continue;
            const i64 cnt = s1 - s0;
            std::unique_ptr<Scratch> vb, tb;
            T* Vc = nullptr;
            T* tc = nullptr;
            if (R.rank == 0) {
                Vc = V2->template as<T>() + s0 * b;
                tc = tau2->template as<T>() + s0;
            } else {
                vb = std::make_unique<Scratch>((size_t)cnt * b * sizeof(T), s);
                tb = std::make_unique<Scratch>((size_t)cnt * sizeof(T), s);
                Vc = vb->template as<T>();
                tc = tb->template as<T>();
            }
            if (P > 1) {
                world->bcast(Vc, (size_t)cnt * b * sizeof(T), 0, s);
                world->bcast(tc, (size_t)cnt * sizeof(T), 0, s);
            }
            if (ncols)
                slate_hip::unmtr_hb2st_blocked_range<K<T>>(n, ncols, kp(static_cast<T*>(SC.buf)), SC.lld, kp(Vc), b,
                                                           kp(tc), spd->as<i64>(), ntd->as<i64>(), nsw, false, Jlo,
                                                           Jhi, s0, s);
            mark();
            NHIP(hipStreamSynchronize(s));
        }
    }
    V2.reset();
    tau2.reset();
    if (stop_at(5)) return 0;
    // ---- Q1 on F's grid, then the caller's layout
    Matrix<T> Zg(n, n, b, p, q);
    redistribute<T>(Zc, Zg);
    Zc = Matrix<T>();
    {
        NTRACE("heev::unmtr_he2hb", s);
        unmtr_he2hb_grid<T>(*F.storage(), pans, *Zg.storage(), s);
    }
    mark();
    redistribute<T>(Zg, *Z);
    g_heev_grid_peak = free0 > low ? free0 - low : 0;
    if (const char* mr = std::getenv("SLATE_AMD_NATIVE_MEMREPORT"); mr && *mr == '1') {
        const double blk = (double)SA.mloc * (double)SA.nloc * sizeof(T);
        std::fprintf(stderr, "rank %d: heev grid %dx%d n=%lld: peak device growth %.1f MB = %.2f x local block "
                     "(%.1f MB); n^2 = %.1f MB\n", R.rank, p, q, (long long)n, g_heev_grid_peak / 1e6,
                     blk > 0 ? g_heev_grid_peak / blk : 0.0, blk / 1e6, (double)n * n * sizeof(T) / 1e6);
    }
    Lambda.assign(w.begin(), w.end());
    return 0;
}

template <typename T>
int64_t heev_impl(HermitianMatrix<T>& A, std::vector<real_t<T>>& Lambda, Matrix<T>* Z) {
    Runtime& R = rt();
    const Storage& SA = *A.storage();
    if (SA.m != SA.n) throw Error("native heev: square matrix");
    const i64 n = SA.n;
    {
        // p x q grids: the distributed solver (no n x n anywhere) unless
        // SLATE_AMD_NATIVE_HEEV=gather (the one-GPU solver behind a gather)
        const bool gather = [] { const char* e = std::getenv("SLATE_AMD_NATIVE_HEEV"); return e && !std::strcmp(e, "gather"); }();
        const bool zok = !Z || (Z->storage()->m == n && Z->storage()->n == n);
        if (R.size > 1 && SA.p * SA.q == R.size && n > 2 * 64 && !gather && zok) return heev_grid<T>(A, Lambda, Z);
    }
    NTRACE("heev", nullptr);
    hipStream_t s = R.main;
    NHIP(hipStreamSynchronize(s));
    if (Z) {
        const Storage& SZ = *Z->storage();
        if (SZ.m != n || SZ.n != n || SZ.p != SA.p || SZ.q != SA.q || SZ.nb != SA.nb)
            throw Error("native heev: Z must be n x n on A's grid and tile size");
    }
    std::vector<double> w((size_t)n, 0.0);
    std::unique_ptr<Scratch> D, Zd;
    int64_t err = 0;
    std::string msg;
    if (R.rank == 0) D = std::make_unique<Scratch>((size_t)std::max<i64>(n, 1) * n * sizeof(T), s);
    gather_root<T>(SA, D ? D->as<T>() : nullptr, s);
    if (R.rank == 0) {
        try {
            symmetrize<T>(n, D->as<T>(), A.uplo(), s);
            if (Z) Zd = std::make_unique<Scratch>((size_t)std::max<i64>(n, 1) * n * sizeof(T), s);
            heev_1gpu<T>(n, D->as<T>(), w, Zd ? Zd->as<T>() : nullptr, Z != nullptr, s);
        } catch (const std::exception& e) {
            err = 1;
            msg = e.what();
        }
    }
    // the eigenvalues (and the error flag) to every rank
    if (R.size > 1) {
        Scratch b((size_t)(n + 1) * sizeof(double), s);
        std::vector<double> h(w);
        h.push_back((double)err);
        upload(b.p, h.data(), h.size() * sizeof(double), s);
        world_comm()->bcast(b.p, h.size() * sizeof(double), 0, s);
        h = download_vec<double>(b.p, h.size(), s);
        err = (int64_t)h.back();
        h.pop_back();
        w = h;
    }
    if (err) {
        if (Z && R.size > 1) {}       // nothing scattered: every rank throws
        throw Error(R.rank == 0 ? msg : std::string("native heev failed on rank 0"));
    }
    if (Z) scatter_root<T>(Zd ? Zd->as<T>() : nullptr, *Z->storage(), s);
    Lambda.assign(w.begin(), w.end());
    return 0;
}

// ---------------------------------------------------------------- SVD
// C -= V op(T) (V^H C), op(T) = T^H (apply Q^H, conj) or T (apply Q)
template <typename T>
void apply_qh(i64 m, i64 kk, const T* V, const T* Tm, T* C, i64 ldc, i64 nc, bool conj, hipStream_t s) {
    if (m <= 0 || nc <= 0 || kk <= 0) return;
    const char ct = ctrans<T>();
    Scratch W((size_t)kk * nc * sizeof(T), s);
    gemm_k<T>(ct, 'N', kk, nc, m, T(1), V, m, C, ldc, T(0), W.as<T>(), kk, s);
    slate_hip::trmm<K<T>>('L', 'U', conj ? ct : 'N', 'N', kk, nc, kv(T(1)), kp(Tm), kk, kp(W.as<T>()), kk, s);
    gemm_k<T>('N', 'N', m, nc, kk, T(-1), V, m, W.as<T>(), kk, T(1), C, ldc, s);
}

// dense m x n (m >= n, ld lda) -> upper band of width nb in place:
// A = Ql B Qr^H (left: column-panel QR reflectors, right: row-panel LQ)
template <typename T>
void ge2tb(i64 m, i64 n, i64 nb, T* A, i64 lda, std::vector<Panel<T>>& left, std::vector<Panel<T>>& right,
           hipStream_t s) {
    const char ct = ctrans<T>();
    for (i64 k0 = 0; k0 < n; k0 += nb) {
        const i64 kb = std::min(nb, n - k0), mp = m - k0, kk = std::min(mp, kb);
        T* P = A + k0 + k0 * lda;
        Panel<T> L;
        L.r0 = k0;
        L.kk = kk;
        L.V = std::make_unique<Scratch>((size_t)mp * kk * sizeof(T), s);
        L.T_ = std::make_unique<Scratch>((size_t)kk * kk * sizeof(T), s);
        {
            Scratch tau((size_t)kk * sizeof(T), s);
            dzero(tau.p, (size_t)kk * sizeof(T), s);
            slate_hip::geqrf_panel_ws<K<T>>(mp, kb, kp(P), lda, kp(tau.as<T>()), kp(L.T_->template as<T>()), kk,
                                            kp(L.V->template as<T>()), mp, rt().qr_work, s);
        }
        if (k0 + kb < n)
            apply_qh<T>(mp, kk, L.V->template as<T>(), L.T_->template as<T>(), A + k0 + (k0 + kb) * lda, lda,
                        n - k0 - kb, true, s);
        zero_strict_lower<T>(mp, kb, P, lda, s);
        left.push_back(std::move(L));
        const i64 c0 = k0 + kb;
        if (c0 >= n) continue;
        const i64 w = n - c0, kr = std::min(w, kb);
        T* X = A + k0 + c0 * lda;                     // kb x w
        Scratch Xh((size_t)w * kb * sizeof(T), s);    // X^H: w x kb
        slate_hip::gecopy<K<T>, K<T>>('G', ct, w, kb, kp(X), lda, kp(Xh.as<T>()), w, s);
        Panel<T> Rt;
        Rt.r0 = c0;
        Rt.kk = kr;
        Rt.V = std::make_unique<Scratch>((size_t)w * kr * sizeof(T), s);
        Rt.T_ = std::make_unique<Scratch>((size_t)kr * kr * sizeof(T), s);
        {
            Scratch tau((size_t)kr * sizeof(T), s);
            dzero(tau.p, (size_t)kr * sizeof(T), s);
            slate_hip::geqrf_panel_ws<K<T>>(w, kb, kp(Xh.as<T>()), w, kp(tau.as<T>()), kp(Rt.T_->template as<T>()),
                                            kr, kp(Rt.V->template as<T>()), w, rt().qr_work, s);
        }
        zero_strict_lower<T>(w, kb, Xh.as<T>(), w, s);
        slate_hip::gecopy<K<T>, K<T>>('G', ct, kb, w, kp(Xh.as<T>()), w, kp(X), lda, s);
        const i64 mr = m - k0 - kb;
        if (mr > 0) {
            // C -= (C V T) V^H on the rows below the panel
            T* C = A + (k0 + kb) + c0 * lda;
            Scratch W((size_t)mr * kr * sizeof(T), s);
            gemm_k<T>('N', 'N', mr, kr, w, T(1), C, lda, Rt.V->template as<T>(), w, T(0), W.as<T>(), mr, s);
            slate_hip::trmm<K<T>>('R', 'U', 'N', 'N', mr, kr, kv(T(1)), kp(Rt.T_->template as<T>()), kr,
                                  kp(W.as<T>()), mr, s);
            gemm_k<T>('N', ct, mr, w, kr, T(-1), W.as<T>(), mr, Rt.V->template as<T>(), w, T(1), C, lda, s);
        }
        right.push_back(std::move(Rt));
    }
}

// one GPU: A (m x n, m >= n, ld m) -> s (descending), U (m x n, ld m) and
// V (n x n, ld n) with A = U diag(s) V^H (wantu / wantv)
template <typename T>
void svd_1gpu(i64 m, i64 n, T* A, std::vector<double>& sv, T* U, T* V, bool wantu, bool wantv, hipStream_t s) {
    using R = real_t<T>;
    const i64 b = std::max<i64>(1, std::min<i64>(64, n));
    std::vector<Panel<T>> left, right;
    ge2tb<T>(m, n, b, A, m, left, right, s);
    // the k x k upper band (0 <= j - i <= b) into a padded working copy
    const i64 k = n, ldp = (k + 7) / 8 * 8 + 72;
    Scratch Bh((size_t)ldp * std::max<i64>(k, 1) * sizeof(T), s);
    {
        slate_hip::TriMask up_, lo_;
        up_.mode = 2;                           // i <= j
        lo_.mode = 1;
        lo_.diag_off = b;                       // i + b >= j
        slate_hip::gecopy_mask<K<T>>(up_, k, k, kp(A), m, kp(Bh.as<T>()), ldp, false, s);
        slate_hip::gecopy_mask<K<T>>(lo_, k, k, kp(Bh.as<T>()), ldp, kp(Bh.as<T>()), ldp, false, s);
    }
    const i64 nsw = std::max<i64>(k - 1, 0);
    std::vector<i64> nt((size_t)std::max<i64>(nsw, 1), 0), sp((size_t)std::max<i64>(k, 1), 0);
    for (i64 j = 0; j < nsw; ++j) {
        const i64 ce0 = std::min(j + b, k - 1);
        nt[j] = 1 + (k - 1 - ce0 + b - 1) / b;
    }
    for (i64 j = 1; j < k; ++j) sp[j] = sp[j - 1] + nt[j - 1];
    const i64 total = nsw ? sp[k - 1] + nt[nsw - 1] : 0, cap = std::max<i64>(total, 1);
    auto store = [&](std::vector<std::unique_ptr<Scratch>>& st) {
        st.push_back(std::make_unique<Scratch>((size_t)cap * b * sizeof(T), s));
        st.push_back(std::make_unique<Scratch>((size_t)cap * sizeof(T), s));
        st.push_back(std::make_unique<Scratch>((size_t)cap * sizeof(i64), s));
        st.push_back(std::make_unique<Scratch>((size_t)cap * sizeof(i64), s));
        dzero(st[0]->p, (size_t)cap * b * sizeof(T), s);
        dzero(st[1]->p, (size_t)cap * sizeof(T), s);
    };
    std::vector<std::unique_ptr<Scratch>> Us, Vs, keep;
    store(Us);
    store(Vs);
    Scratch* ntd = upload_vec(keep, nt, s);
    Scratch* spd = upload_vec(keep, sp, s);
    if (nsw > 0) {
        Scratch work((size_t)(nsw + 2) * sizeof(int), s);
        dzero(work.p, (size_t)(nsw + 2) * sizeof(int), s);
        hipDeviceProp_t pr;
        NHIP(hipGetDeviceProperties(&pr, rt().device));
        const i64 nt0 = nt[0] ? nt[0] : 1;
        const int nwg = (int)std::min<i64>({std::max<i64>(nsw, 1), (i64)pr.multiProcessorCount,
                                            std::max<i64>(8, nt0 / 4 + 8)});
        slate_hip::tb2bd_device<K<T>>(k, (int)b, kp(Bh.as<T>()), ldp, kp(Us[0]->as<T>()), kp(Us[1]->as<T>()),
                                      Us[2]->as<i64>(), Us[3]->as<i64>(), kp(Vs[0]->as<T>()), kp(Vs[1]->as<T>()),
                                      Vs[2]->as<i64>(), Vs[3]->as<i64>(), spd->as<i64>(), ntd->as<i64>(),
                                      work.as<int>(), nsw, nwg, s);
    }
    // diagonal / super-diagonal, and the phases of a complex bidiagonal
    Scratch dsub((size_t)2 * std::max<i64>(k, 1) * sizeof(T), s);
    copy2d(dsub.as<T>(), 1, Bh.as<T>(), ldp + 1, 1, k, s);
    if (k > 1) copy2d(dsub.as<T>() + k, 1, Bh.as<T>() + ldp, ldp + 1, 1, k - 1, s);
    const std::vector<T> ds = download_vec<T>(dsub.p, (size_t)(2 * k), s);
    std::vector<double> d((size_t)k), e((size_t)std::max<i64>(k, 1), 0.0);
    std::vector<T> pu((size_t)k, T(1)), pv((size_t)k, T(1));
    for (i64 i = 0; i < k; ++i) {
        if constexpr (is_cplx<T>()) {
            const T x = ds[i] * pv[i];
            const R ax = std::abs(x);
            pu[i] = ax > R(0) ? x / ax : T(1);
            d[i] = (double)ax;
            if (i < k - 1) {
                const T y = std::conj(pu[i]) * ds[k + i];
                const R ay = std::abs(y);
                pv[i + 1] = ay > R(0) ? std::conj(y / ay) : T(1);
                e[i] = (double)ay;
            }
        } else {
            d[i] = (double)ds[i];
            if (i < k - 1) e[i] = (double)ds[k + i];
        }
    }
    std::vector<double> Uh(wantu ? (size_t)k * k : 0, 0.0), VTh(wantv ? (size_t)k * k : 0, 0.0);
    for (i64 i = 0; i < k && wantu; ++i) Uh[i + i * k] = 1.0;
    for (i64 i = 0; i < k && wantv; ++i) VTh[i + i * k] = 1.0;
    if (slate_tridiag::bdsqr_impl(k, d.data(), e.data(), wantu ? Uh.data() : nullptr, k, wantu ? k : 0,
                                  wantv ? VTh.data() : nullptr, k, wantv ? k : 0))
        throw Error("native svd: the bidiagonal QR iteration did not converge");
    sv = d;
    auto back = [&](std::vector<std::unique_ptr<Scratch>>& F, const std::vector<double>& Qh, const std::vector<T>& ph,
                    T* Z, i64 ldz, std::vector<Panel<T>>& panels) {
        Scratch* q = upload_vec(keep, Qh, s);
        Scratch* phd = is_cplx<T>() ? upload_vec(keep, ph, s) : nullptr;
        real_to_phase<T>(k, k, q->as<double>(), k, phd ? kp(phd->as<T>()) : nullptr, kp(Z), ldz, s);
        if (nsw > 0 &&
            !slate_hip::unmtr_hb2st_blocked<K<T>>(k, k, kp(Z), ldz, kp(F[0]->as<T>()), b, kp(F[1]->as<T>()),
                                                  spd->as<i64>(), ntd->as<i64>(), nsw, false, s)) {
            for (i64 j = k - 1; j >= 0; --j) {
                const i64 first = sp[j], last = j + 1 < k ? sp[j + 1] : total;
                if (last > first)
                    slate_hip::apply_refl_batch<K<T>>(k, kp(Z), ldz, kp(F[0]->as<T>()), b, kp(F[1]->as<T>()),
                                                      F[2]->as<i64>(), F[3]->as<i64>(), first, last - first, false, s);
            }
        }
        for (auto it = panels.rbegin(); it != panels.rend(); ++it) {
            const i64 mr = (&panels == &left ? m : k) - it->r0;
            apply_qh<T>(mr, it->kk, it->V->template as<T>(), it->T_->template as<T>(), Z + it->r0, ldz, k, false, s);
        }
    };
    if (wantu) {
        dzero(U, (size_t)m * k * sizeof(T), s);
        back(Us, Uh, pu, U, m, left);
    }
    if (wantv) {
        std::vector<double> Vh((size_t)k * k);                 // V = VT^T (real)
        for (i64 j = 0; j < k; ++j)
            for (i64 i = 0; i < k; ++i) Vh[i + j * k] = VTh[j + i * k];
        back(Vs, Vh, pv, V, k, right);
    }
    NHIP(hipStreamSynchronize(s));
}

template <typename T>
int64_t svd_impl(Matrix<T>& A, std::vector<real_t<T>>& S, Matrix<T>* U, Matrix<T>* VH) {
    NTRACE("svd", nullptr);
    Runtime& R = rt();
    const Storage& SA = *A.storage();
    const i64 m0 = SA.m, n0 = SA.n, k = std::min(m0, n0);
    hipStream_t s = R.main;
    NHIP(hipStreamSynchronize(s));
    if (U) {
        const Storage& SU = *U->storage();
        if (SU.m != m0 || SU.n != k || SU.p != SA.p || SU.q != SA.q || SU.nb != SA.nb)
            throw Error("native svd: U must be m x min(m, n) on A's grid and tile size");
    }
    if (VH) {
        const Storage& SV = *VH->storage();
        if (SV.m != k || SV.n != n0 || SV.p != SA.p || SV.q != SA.q || SV.nb != SA.nb)
            throw Error("native svd: VH must be min(m, n) x n on A's grid and tile size");
    }
    std::vector<double> sv((size_t)k, 0.0);
    std::unique_ptr<Scratch> D, Du, Dv;
    int64_t err = 0;
    std::string msg;
    if (R.rank == 0) D = std::make_unique<Scratch>((size_t)std::max<i64>(m0 * n0, 1) * sizeof(T), s);
    gather_root<T>(SA, D ? D->as<T>() : nullptr, s);
    if (R.rank == 0 && k > 0) {
        try {
            const bool tr = m0 < n0;             // factor A^H = V S U^H when wide
            const i64 m = tr ? n0 : m0, n = tr ? m0 : n0;
            Scratch At((size_t)m * n * sizeof(T), s);
            if (tr) slate_hip::gecopy<K<T>, K<T>>('G', ctrans<T>(), m, n, kp(D->as<T>()), m0, kp(At.as<T>()), m, s);
            else copy2d(At.as<T>(), m, D->as<T>(), m0, m, n, s);
            const bool wu = tr ? VH != nullptr : U != nullptr, wv = tr ? U != nullptr : VH != nullptr;
            Scratch Zu((size_t)(wu ? m * n : 1) * sizeof(T), s), Zv((size_t)(wv ? n * n : 1) * sizeof(T), s);
            svd_1gpu<T>(m, n, At.as<T>(), sv, Zu.as<T>(), Zv.as<T>(), wu, wv, s);
            // outputs of op(A): not transposed U = Zu (m x k), VH = Zv^H;
            // transposed U = Zv (k x k), VH = Zu^H (k x n0)
            if (U) {
                Du = std::make_unique<Scratch>((size_t)m0 * k * sizeof(T), s);
                if (tr) copy2d(Du->as<T>(), m0, Zv.as<T>(), n, m0, k, s);
                else copy2d(Du->as<T>(), m0, Zu.as<T>(), m, m0, k, s);
            }
            if (VH) {
                Dv = std::make_unique<Scratch>((size_t)k * n0 * sizeof(T), s);
                if (tr) slate_hip::gecopy<K<T>, K<T>>('G', ctrans<T>(), k, n0, kp(Zu.as<T>()), m, kp(Dv->as<T>()), k, s);
                else slate_hip::gecopy<K<T>, K<T>>('G', ctrans<T>(), k, n0, kp(Zv.as<T>()), n, kp(Dv->as<T>()), k, s);
            }
            NHIP(hipStreamSynchronize(s));
        } catch (const std::exception& e) {
            err = 1;
            msg = e.what();
        }
    }
    if (R.size > 1) {
        Scratch bb((size_t)(k + 1) * sizeof(double), s);
        std::vector<double> h(sv);
        h.push_back((double)err);
        upload(bb.p, h.data(), h.size() * sizeof(double), s);
        world_comm()->bcast(bb.p, h.size() * sizeof(double), 0, s);
        h = download_vec<double>(bb.p, h.size(), s);
        err = (int64_t)h.back();
        h.pop_back();
        sv = h;
    }
    if (err) throw Error(R.rank == 0 ? msg : std::string("native svd failed on rank 0"));
    if (U) scatter_root<T>(Du ? Du->as<T>() : nullptr, *U->storage(), s);
    if (VH) scatter_root<T>(Dv ? Dv->as<T>() : nullptr, *VH->storage(), s);
    S.assign(sv.begin(), sv.end());
    return 0;
}

}  // namespace

template <typename T>
int64_t svd(Matrix<T>& A, std::vector<real_t<T>>& S, Matrix<T>& U, Matrix<T>& VH, const Options&) {
    return svd_impl<T>(A, S, &U, &VH);
}
template <typename T>
int64_t svd(Matrix<T>& A, std::vector<real_t<T>>& S, const Options&) {
    return svd_impl<T>(A, S, nullptr, nullptr);
}

template <typename T>
int64_t heev(HermitianMatrix<T>& A, std::vector<real_t<T>>& Lambda, Matrix<T>& Z, const Options&) {
    return heev_impl<T>(A, Lambda, &Z);
}
template <typename T>
int64_t heev(HermitianMatrix<T>& A, std::vector<real_t<T>>& Lambda, const Options&) {
    return heev_impl<T>(A, Lambda, nullptr);
}

#define SLATE_NATIVE_EIG_INST(T)                                                                            \
    template int64_t heev<T>(HermitianMatrix<T>&, std::vector<real_t<T>>&, Matrix<T>&, const Options&);    \
    template int64_t heev<T>(HermitianMatrix<T>&, std::vector<real_t<T>>&, const Options&);                \
    template int64_t svd<T>(Matrix<T>&, std::vector<real_t<T>>&, Matrix<T>&, Matrix<T>&, const Options&);  \
    template int64_t svd<T>(Matrix<T>&, std::vector<real_t<T>>&, const Options&);
SLATE_NATIVE_EIG_INST(float)
SLATE_NATIVE_EIG_INST(double)
SLATE_NATIVE_EIG_INST(std::complex<float>)
SLATE_NATIVE_EIG_INST(std::complex<double>)
#undef SLATE_NATIVE_EIG_INST

}  // namespace native
}  // namespace slate_amd
