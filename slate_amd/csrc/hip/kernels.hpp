// Declarations of the non-GEMM gfx950 kernel launchers (see the .hip files).
#pragma once
#include "common.hpp"

namespace slate_hip {

template <typename T> void potrf_tile(char uplo, int n, T* A, i64 lda, i64* info, hipStream_t s);
template <typename T>
void trsm(char side, char uplo, char trans, char diag, i64 m, i64 n, T alpha,
          const T* A, i64 lda, T* B, i64 ldb, hipStream_t s);
template <typename T>
void trmm(char side, char uplo, char trans, char diag, i64 m, i64 n, T alpha,
          const T* A, i64 lda, T* B, i64 ldb, hipStream_t s);

// chol_fast.hip (fp64 fast paths; return false when the shape is not covered)
bool potrf_fast(int n, double* A, i64 lda, i64* info, i64 info_off, hipStream_t s, const int* gate = nullptr,
                const double* floorp = nullptr);
void potrf_lds_profile(int n, double* A, i64 lda, i64* info, i64* prof, hipStream_t s);
// potrf_mc.hip: multi-workgroup 64-blocked tile Cholesky (n <= 512)
bool potrf_mc(int n, double* A, i64 lda, i64* info, i64 info_off, hipStream_t s, const int* gate = nullptr,
              const double* floorp = nullptr);
void potrf_mc_set_prof(i64* prof);
bool potrf_lds(int n, double* A, i64 lda, i64* info, i64 info_off, hipStream_t s, const int* gate = nullptr,
               const double* floorp = nullptr);
bool trsm_rlt_fast(i64 m, i64 n, double alpha, const double* L, i64 ldl, double* B, i64 ldb, bool unit,
                   hipStream_t s, const int* gate = nullptr);
bool trsm_lln_fast(i64 m, i64 n, double alpha, const double* L, i64 ldl, double* B, i64 ldb, bool unit,
                   hipStream_t s);
// qr_fast.hip: tall fp64 QR panel (CholeskyQR2, device-decided fallback to a
// perturbed shifted CholeskyQR3, Householder reconstruction); false = not
// applicable (shape / SLATE_AMD_QR_PANEL=householder).  No host read-back.
bool geqrf_cholqr(i64 m, i64 b, double* A, i64 lda, double* tau, double* Tm, i64 ldt, double* V, i64 ldv,
                  hipStream_t s);

// aux.hip
template <typename T> void geset(char uplo, i64 m, i64 n, T off, T diag, T* A, i64 lda, hipStream_t s);
template <typename T> void gescale(char uplo, i64 m, i64 n, T alpha, T* A, i64 lda, hipStream_t s);
template <typename T>
void geadd(char uplo, i64 m, i64 n, T alpha, const T* A, i64 lda, T beta, T* B, i64 ldb, hipStream_t s);
template <typename Ts, typename Td>
void gecopy(char uplo, char trans, i64 m, i64 n, const Ts* A, i64 lda, Td* B, i64 ldb, hipStream_t s);
template <typename T>
void gecopy_mask(const TriMask& mk, i64 m, i64 n, const T* A, i64 lda, T* B, i64 ldb, bool real_diag,
                 hipStream_t s);
// the same, B unchanged outside the mask
template <typename T>
void gecopy_mask_merge(const TriMask& mk, i64 m, i64 n, const T* A, i64 lda, T* B, i64 ldb, hipStream_t s);
template <typename T, typename R>
void butterfly(bool trans, bool rows, int depth, i64 nidx, i64 nother, T* A, i64 lda, const R* diag, i64 ldd,
               hipStream_t s);
template <typename T, typename R>
void gescale_row_col(char equed, i64 m, i64 n, const R* r, const R* c, T* A, i64 lda, hipStream_t s);
template <typename T>
void laswp(i64 n, T* A, i64 lda, i64 k1, i64 k2, const i64* ipiv, int incx, hipStream_t s);
template <typename T>
void permute_rows_scatter(i64 m, i64 n, const T* A, i64 lda, T* B, i64 ldb, const i64* perm, hipStream_t s);
void spin_ns(double ns, hipStream_t s);   // aux.hip: hold the stream for ns (loopback link model)
template <typename T>
void permute_rows_gather(i64 m, i64 n, const T* A, i64 lda, T* B, i64 ldb, const i64* perm, hipStream_t s);

// distributed row interchange (aux.hip): device-resident swap plan, owner-masked
// pack/unpack around one column all-reduce; CALU selection -> LAPACK ipiv
void swap_plan(i64 k1, i64 k2, const i64* ipiv, i64 ioff, int incx, void* plan, hipStream_t s);
size_t swap_plan_bytes();
template <typename T>
void xchg_gather(const void* plan, i64 S, i64 n, const T* A, i64 lda, T* X, i64 ldx, i64 nb, int p, int pr,
                 hipStream_t s);
template <typename T>
void xchg_scatter(const void* plan, i64 S, i64 n, const T* X, i64 ldx, T* A, i64 lda, i64 nb, int p, int pr,
                  hipStream_t s);
void sel_to_ipiv(const i64* sel, i64 kb, i64 r0, i64* ipiv, hipStream_t s);

// norm.hip: kind 'M' max, '1' one (column sums), 'I' inf (row sums), 'F' fro
// (scale/sumsq pairs -> here plain sum of squares with scaling by the max);
// out receives per-column (one), per-row (inf) or a single value.
template <typename T, typename R>
void genorm(char norm, char uplo, char diag, int herm, i64 m, i64 n, const T* A, i64 lda, R* out,
            hipStream_t s);

// getrf.hip
template <typename T>
void getrf_panel_ws(i64 m, i64 n, T* A, i64 lda, i64* ipiv, i64* info, double thr, bool nopiv,
                    void* work, hipStream_t s);
size_t getrf_work_bytes();
void lu_persist_profile(int enable, unsigned long long* out);
unsigned long long lu_persist_fallbacks(int force);
template <typename T>
void laswp_off(i64 n, T* A, i64 lda, i64 k1, i64 k2, const i64* ipiv, i64 ioff, hipStream_t s, int incx = 1);
template <typename T>
void laswp_cols(i64 nrows, T* A, i64 lda, i64 k1, i64 k2, const i64* ipiv, i64 ioff, hipStream_t s, int incx = 1);
template <typename T>
void laswp_cols_plan(i64 nrows, T* A, i64 lda, const void* plan, hipStream_t s);

// lu_dist.hip: one column step of the distributed partial-pivoting panel
template <typename T>
void lu_dist_step(i64 nr, T* W, i64 ldw, const i64* grow, int c0, int c1, int j, const T* recs, int p, T* Tt,
                  i64 ldt, i64* ipiv, i64* info, i64 info_off, double thr, T* rec, void* part, i64 diag_local,
                  hipStream_t s);

// lu_dist.hip: device-resident b-column base block of the same panel; the
// column peers exchange their records through peer-mapped mailboxes
struct LuPeer {
    const unsigned long long* mbox;  // device array [p]: mailbox base of each column peer (mbox[me] = own)
    int p, me;
    char* part;                      // this rank's partial slots (lu_peer_part_bytes, zeroed once)
    long long seq0;                  // host sequence number: column j of the call tags seq0 + (j - c0) + 1
    int has_diag;                    // this rank holds the panel's top rows (local row j = panel row j)
    unsigned long long* err;         // set non-zero on a timed-out wait
};
size_t lu_peer_mailbox_bytes();
size_t lu_peer_part_bytes();
int lu_peer_max_b();
int lu_peer_max_p();
void* lu_peer_alloc(size_t bytes, void* handle64);
void* lu_peer_open(const void* handle64);
void lu_peer_close(void* p);
void lu_peer_free(void* p);
template <typename T>
void lu_dist_base(i64 nr, T* W, i64 ldw, const i64* grow, int c0, int c1, T* Tt, i64 ldt, i64* ipiv, i64* info,
                  i64 info_off, double thr, const LuPeer& pe, int G, hipStream_t s);

// geqrf.hip
template <typename T>
void geqrf_panel_ws(i64 m, i64 n, T* A, i64 lda, T* tau, T* Tm, i64 ldt, T* V, i64 ldv, void* work,
                    hipStream_t s);
size_t geqrf_work_bytes();
// tpqrt.hip
template <typename T>
void tpqrt_panel(i64 m, i64 l, i64 j0, int ib, T* A, i64 lda, T* B, i64 ldb, T* V, i64 ldv, T* tau, T* Tm,
                 i64 ldt, hipStream_t s);
template <typename T>
void hb2st_device(i64 n, int b, T* A, i64 lda, T* V, T* tau, i64* row, i64* len, const i64* sweep_ptr,
                  const i64* ntask, int* work, i64 nsw, int nwg, hipStream_t s, i64* prof = nullptr,
                  i64 extent = 0);   // elements of A addressed (0: lda n; a skewed band layout passes its own)
template <typename T>
void tb2bd_device(i64 n, int b, T* A, i64 lda, T* UV, T* Utau, i64* Urow, i64* Ulen, T* VV, T* Vtau, i64* Vrow,
                  i64* Vlen, const i64* sweep_ptr, const i64* ntask, int* work, i64 nsw, int nwg, hipStream_t s);
template <typename T>
void apply_refl_batch(i64 ncols, T* Z, i64 ldz, const T* V, i64 b, const T* tau, const i64* row, const i64* len,
                      i64 first, i64 count, bool conj_tau, hipStream_t s);
template <typename T>
bool unmtr_hb2st_blocked(i64 n, i64 ncols, T* Z, i64 ldz, const T* V, i64 b, const T* tau, const i64* sp,
                         const i64* nt, i64 nsw, bool conj_tau, hipStream_t s);
// sweep blocks [Jlo, Jhi] of b sweeps only, V / tau holding the slots from
// slot0 on (a streamed chunk of the reflectors)
template <typename T>
bool unmtr_hb2st_blocked_range(i64 n, i64 ncols, T* Z, i64 ldz, const T* V, i64 b, const T* tau, const i64* sp,
                               const i64* nt, i64 nsw, bool conj_tau, i64 Jlo, i64 Jhi, i64 slot0, hipStream_t s);
bool unmtr_hb2st_mfma(i64 n, i64 ncols, double* Z, i64 ldz, const double* V, i64 b, const double* tau,
                      const i64* sp, const i64* nt, const i64* gJ, const i64* gt, const i64* gptr, i64 ngroups,
                      double* Tg, i64 nsw, hipStream_t s, int phase = 3);
template <typename T> void v_explicit(i64 m, i64 n, const T* A, i64 lda, T* V, i64 ldv, hipStream_t s);
template <typename T> void trtri(char uplo, char diag, i64 n, T* A, i64 lda, i64* info, hipStream_t s);
template <typename T> void tri_inv(char uplo, char diag, i64 n, const T* A, i64 lda, T* W, i64 ldw, hipStream_t s);

// stedc.hip
// device-resident merges of one D&C tree level (stedc_level_prep: sort,
// deflation, Givens runs, compacted index sets; meta = MergeMeta per merge)
void stedc_level_prep(i64 n, i64 nm, i64 maxs, const i64* desc, const double* rho, const double* W, const double* Z,
                      double* dd, double* zs, int* ty, i64* order, i64* c, int* keep, int* rot, double* cs,
                      double* sn, void* meta, i64* K, i64* S1, i64* KS1, i64* S2, i64* KS2, i64* D, i64* isK,
                      i64* rI, i64* rJ, double* rC, double* rS, hipStream_t s);
size_t stedc_meta_bytes();
void stedc_lambda(i64 s, const double* dd, const i64* isK, const double* dK, const i64* org, const double* mu,
                  int flip, double* lam, hipStream_t st);
void stedc_merge2(const double* lam, const i64* L1, i64 n1, const i64* L2, i64 n2, int rev, i64* out,
                  hipStream_t st);
void cols_copy(i64 m, i64 nc, const double* A, i64 lda, const i64* idx, double* B, i64 ldb, bool scatter,
               hipStream_t st);
void vec_gather(i64 n, const double* x, const i64* idx, double* y, hipStream_t st);
void stedc_secular(i64 n, const double* d, const double* z, double rho, double zz, i64* org, double* mu,
                   double* zh, double* V, i64 ldv, hipStream_t s);
void steqr_leaves(i64 nleaf, const i64* lo, const i64* hi, const double* d, const double* e, double* w, double* Q,
                  i64 ldq, i64 r0, i64 r1, i64* fails, hipStream_t s, int maxleaf, int maxit = 60);
void stedc_runs(i64 nn, const i64* c, const double* dd, double* z, int* ty, double tol, double* cs, double* sn,
                int* rot, int* keep, hipStream_t s);
void rot_cols(i64 m, double* Q, i64 ldq, i64 nrot, const i64* I, const i64* J, const double* C, const double* S,
              hipStream_t s);
void stedc_vectors(i64 n, const double* d, const double* zh, const i64* org, const double* mu, i64 j0, i64 nc,
                   double* V, i64 ldv, hipStream_t s);

// matgen.hip
template <typename T>
void matgen(int kind, uint64_t seed, i64 mloc, i64 nloc, T* A, i64 lda, i64 m, i64 n,
            i64 mb, int p, int pr, i64 nb, int q, int pc, i64 row0, i64 col0, double scale, hipStream_t s);

}  // namespace slate_hip
