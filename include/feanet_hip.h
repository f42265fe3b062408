/*
 * feanet_hip.h — C ABI of libfeanet_hip.so, the MI355X (gfx950) kernels of the
 * FEANet geometric-multigrid hot path.
 *
 * The reference (longfish/Multigrid-FEANet) has no native code: its hot path is
 * PyTorch-CPU conv2d / conv_transpose2d inside nn.Modules.  Each entry point below
 * replaces one of those module methods; the reference interface it stands in for is
 * cited per function.  Python binds them with ctypes (feanet_amd/_lib.py); the
 * reference-side binding a maintainer would add is shown in INTEGRATION.md.
 *
 * Conventions
 *  - T is float (suffix _f32) or double (suffix _f64); arithmetic stays in T.
 *  - All data pointers are DEVICE pointers owned by the caller; calls are
 *    asynchronous on `stream` (a hipStream_t passed as void*; NULL = default).
 *  - Return value: 0 on success, FEA_EINVAL (-1) for invalid arguments (nothing is
 *    launched), otherwise the hipError_t of the launch.  No exception crosses the ABI.
 *  - Functions are stateless and re-entrant; they never allocate or synchronise,
 *    so they are safe inside hipGraph stream capture.
 *  - Stencil tables: `ktab` = ntab x 9 coefficients (row-major 3x3, cross-correlation
 *    orientation, ktab[p*9 + 3*dr + dc] multiplies u[r+dr-1][c+dc-1]); `omd` = ntab
 *    values omega/d_p (d_p = ktab[p*9+4]); `pid` = uint8 pattern id per node (NULL:
 *    every node uses pattern 0).  ntab <= FEA_MAX_PATTERNS.
 *
 * Two families:
 *  (1) "Generic" ops on contiguous NCHW tensors [B, C, H, W] — the drop-in operator
 *      boundary used by the FEANet.* shim modules (KNet/FNet/JacobiBlock/MultiGrid).
 *  (2) "mg" ops on FRAMED level buffers owned by the MultigridSolver: node (r, c)
 *      of sample b lives at  base[b*bstride + (r+1)*ld + (A-1) + c],  A = 128/sizeof(T)
 *      (so column 1 starts a 128-byte line), with a ghost ring at r = -1, H and c = -1, W.
 *      Use fea_mg_layout() for ld / bstride.  Boundary nodes hold the Dirichlet values
 *      and are never written by mg kernels (SURVEY §8a A9 invariant).
 */
#ifndef FEANET_HIP_H
#define FEANET_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FEA_EINVAL (-1)
#define FEA_MAX_PATTERNS 16

/* ---------------------------------------------------------------------------
 * Library / layout queries
 * ------------------------------------------------------------------------- */
/* ABI version (bumped on any signature change; 2 = H x W framed grids, 3 = fused residual norms of
 * fea_mg_cycle_join / fea_mg_sweep_restrict). */
int fea_abi_version(void);

/* Framed layout of an H x W level for elements of `elem_size` bytes (4 or 8):
 * writes the row pitch (elements) and the per-sample stride (elements).
 * Returns 0, or FEA_EINVAL for unsupported H, W / elem_size. */
int fea_mg_layout(int H, int W, int elem_size, int* ld, long long* bstride);

/* Bytes of double workspace needed by the norm kernels for this shape. */
size_t fea_norm_workspace_bytes(int B, int H, int W);

/* Fused residual norms, deferred: fea_mg_cycle_join with norm_ws != NULL and norm_hist == NULL only
 * writes its per-wave partial sums of squares, fea_mg_join_norm_parts(B, H, W, elem_size) per sample
 * (sample b at norm_ws[b * per ..]); fea_norm_append then reduces nrows such partial sets (set r at
 * ws + r * stride, stride >= B * per doubles) in index order and appends sqrt as rows cnt[1] ..
 * cnt[1] + nrows - 1 of hist (B doubles per row), cnt[1] += nrows.  A solve loop gives each joined cycle
 * of a graph block its own partial set and reduces them with ONE launch at the block's end. */
long long fea_mg_join_norm_parts(int B, int H, int W, int elem_size);
int fea_norm_append(const double* ws, long long stride, long long per, int B, int nrows, double* hist,
                    unsigned* cnt, void* stream);

/* ---------------------------------------------------------------------------
 * (1) Generic ops, contiguous [B, C, H, W]
 * ------------------------------------------------------------------------- */

/* y = K u: y[i] = sum_d ktab[pid(i+d)][d] * u[i+d], zero padding.
 * Replaces KNet.forward (FEANet/model.py:22-30); with ntab=1, pid=NULL it is FNet.forward
 * (model.py:60-61) and one HNet layer (M-FEANet-mg_test.ipynb:104-106) too.  pid is [H, W]. */
int fea_knet_apply_f32(const float* u, float* y, const uint8_t* pid, const float* ktab, int ntab,
                       int B, int H, int W, void* stream);
int fea_knet_apply_f64(const double* u, double* y, const uint8_t* pid, const double* ktab, int ntab,
                       int B, int H, int W, void* stream);

/* xs[b, p] = (pid == p) ? x[b] : 0, p < C.  Replaces KNet.split_x (model.py:37-47). */
int fea_split_x_f32(const float* x, float* xs, const uint8_t* pid, int C, int B, int H, int W, void* stream);
int fea_split_x_f64(const double* x, double* xs, const uint8_t* pid, int C, int B, int H, int W, void* stream);

/* Periodic weighted-Jacobi sweep (JacobiBlockPBC.jacobi_convolution, FEANet/jacobi.py:86-97), period
 * n = N - 1, single pattern: out (B x N x N) = omd[0] * (f(a+1, b+1) - K u_periodic(a, b)) +
 * u(a mod n, b mod n); f is the (N+2) x (N+2) forcing term (FNet of the periodic extension). */
int fea_jacobi_sweep_pbc_f32(const float* u, const float* f, float* out, const float* ktab, const float* omd,
                             int B, int N, void* stream);
int fea_jacobi_sweep_pbc_f64(const double* u, const double* f, double* out, const double* ktab,
                             const double* omd, int B, int N, void* stream);
/* Circular extension of u[:, :-1, :-1] (period N - 1) to (N - 1 + lo + hi)^2 (lo rows/columns before):
 * pbc_boundary (jacobi.py:72-79) is lo = 1, hi = 2; reset_boundary (:81-84) is lo = 0, hi = 1. */
int fea_pbc_pad_f32(const float* u, float* dst, int B, int N, int lo, int hi, void* stream);
int fea_pbc_pad_f64(const double* u, double* dst, int B, int N, int lo, int hi, void* stream);

/* One weighted-Jacobi sweep, out-of-place:
 *   u0 = u*geo + bc; r = f - K u0; out = (omd[pid]*r + u0)*geo + bc.
 * geo/bc: NULL = square domain (1 inside, 0 on the edge) / zero; *_bstride = elements
 * between samples (0 = broadcast).  Replaces JacobiBlock.jacobi_convolution
 * (FEANet/jacobi.py:39-47) with reset_boundary (:27-29) fused in. */
int fea_jacobi_sweep_f32(const float* u, const float* f, float* out, const uint8_t* pid,
                         const float* ktab, const float* omd, int ntab,
                         const float* geo, long long geo_bstride, const float* bc, long long bc_bstride,
                         int B, int H, int W, void* stream);
int fea_jacobi_sweep_f64(const double* u, const double* f, double* out, const uint8_t* pid,
                         const double* ktab, const double* omd, int ntab,
                         const double* geo, long long geo_bstride, const double* bc, long long bc_bstride,
                         int B, int H, int W, void* stream);

/* r = f - K u (the residual every driver forms, e.g. FEANet/multigrid.py:168). */
int fea_residual_f32(const float* u, const float* f, float* r, const uint8_t* pid, const float* ktab,
                     int ntab, int B, int H, int W, void* stream);
int fea_residual_f64(const double* u, const double* f, double* r, const uint8_t* pid, const double* ktab,
                     int ntab, int B, int H, int W, void* stream);

/* Restriction, H = W = 2^k + 1 fine nodes -> Hc = (H+1)/2:
 *   fc = w0 * pad0( conv2d(x[..., 1:-1, 1:-1], rtab, stride 2) ).
 * C > 1: x is the split field [B, C, H, W], rtab holds C channel kernels (pid ignored).
 * C == 1: x is [B, 1, H, W] and the kernel of each fine node is rtab[pid(node)].
 * Replaces RestrictionNet.forward + MultiGrid.Restrict (FEANet/multigrid.py:50-60,115-122)
 * and the mg_test / MM notebook Restrict methods. */
int fea_restrict_f32(const float* x, int C, float* fc, const uint8_t* pid, const float* rtab, int ntab,
                     float w0, int B, int H, int W, void* stream);
int fea_restrict_f64(const double* x, int C, double* fc, const uint8_t* pid, const double* rtab, int ntab,
                     double w0, int B, int H, int W, void* stream);

/* Prolongation, coarse Hc x Wc -> fine (2Hc-1) x (2Wc-1):
 *   out = add + w1 * conv_transpose2d(e, ptab, stride 2, padding 1)      (add may be NULL)
 * C > 1: e is split [B, C, Hc, Wc]; C == 1: kernel of coarse node = ptab[pidc(node)].
 * Replaces ProlongationNet.forward + MultiGrid.Interpolate (FEANet/multigrid.py:62-73,124-130)
 * and the `v + eF_delta` update (:179-180). */
int fea_prolong_f32(const float* e, int C, float* out, const float* add, const uint8_t* pidc,
                    const float* ptab, int ntab, float w1, int B, int Hc, int Wc, void* stream);
int fea_prolong_f64(const double* e, int C, double* out, const double* add, const uint8_t* pidc,
                    const double* ptab, int ntab, double w1, int B, int Hc, int Wc, void* stream);

/* out[b] = || r[b, 0, 1:-1, 1:-1] ||_2 with r = f - K u (u may be the residual itself: pass
 * f = NULL and ktab = NULL to take the norm of u).  Deterministic two-pass reduction; ws must
 * hold fea_norm_workspace_bytes(B, H, W) bytes.  Replaces the drivers'
 * torch.norm(residual[:, :, 1:-1, 1:-1], dim=(2,3)) (M-FEANet-mg_test.ipynb:27428-27429). */
int fea_residual_norm_f32(const float* u, const float* f, const uint8_t* pid, const float* ktab, int ntab,
                          double* out, double* ws, int B, int H, int W, void* stream);
int fea_residual_norm_f64(const double* u, const double* f, const uint8_t* pid, const double* ktab, int ntab,
                          double* out, double* ws, int B, int H, int W, void* stream);

/* Adjoints of the generic ops, for autograd through the reference's training forward
 * (MultiGrid.forward / qm, FEANet/multigrid.py:132-157; the reference gets them from torch's
 * conv2d / conv_transpose2d backward).  Same layouts and argument meaning as the forward ops;
 * g is the gradient of the forward op's output.
 *   knet_apply_adj:   out = K^T g                 ((K^T g)[j] = sum_d ktab[pid(j)][d] g[j - d])
 *   jacobi_sweep_adj: gf = omd . geo . g,  gu = geo . (geo . g - K^T gf)   (gf may be NULL)
 *   restrict_adj:     gx = d fc / d x   applied to g  (g [B, 1, Hc, Wc] -> gx [B, C, H, W])
 *   prolong_adj:      ge = d out / d e  applied to g  (g [B, 1, H, W]  -> ge [B, C, Hc, Wc])
 *   transfer_weight_grad: gw[ch][k] = scale * sum_{(a, b)} cf[ch_c][a][b] * ff[ch_f][2a-1+ky][2b-1+kx],
 *     (a, b) over the coarse interior (interior = 1, restriction) or all coarse nodes (0,
 *     prolongation); ch_c = ch when c_split else 0, ch_f likewise; gw is [C, 9]; ws holds
 *     fea_transfer_weight_grad_ws_bytes(C, B, Hc, Wc) bytes; fixed-order (deterministic) sums.
 *     Restriction weights: cf = g, ff = x (split).  Prolongation weights: cf = e (split), ff = g. */
int fea_knet_apply_adj_f32(const float* g, float* out, const uint8_t* pid, const float* ktab, int ntab,
                           int B, int H, int W, void* stream);
int fea_knet_apply_adj_f64(const double* g, double* out, const uint8_t* pid, const double* ktab, int ntab,
                           int B, int H, int W, void* stream);
int fea_jacobi_sweep_adj_f32(const float* g, float* gu, float* gf, const uint8_t* pid, const float* ktab,
                             const float* omd, int ntab, const float* geo, long long geo_bs, int B, int H,
                             int W, void* stream);
int fea_jacobi_sweep_adj_f64(const double* g, double* gu, double* gf, const uint8_t* pid,
                             const double* ktab, const double* omd, int ntab, const double* geo,
                             long long geo_bs, int B, int H, int W, void* stream);
int fea_restrict_adj_f32(const float* g, int C, float* gx, const uint8_t* pid, const float* rtab, int ntab,
                         float w0, int B, int H, int W, void* stream);
int fea_restrict_adj_f64(const double* g, int C, double* gx, const uint8_t* pid, const double* rtab,
                         int ntab, double w0, int B, int H, int W, void* stream);
int fea_prolong_adj_f32(const float* g, int C, float* ge, const uint8_t* pidc, const float* ptab, int ntab,
                        float w1, int B, int Hc, int Wc, void* stream);
int fea_prolong_adj_f64(const double* g, int C, double* ge, const uint8_t* pidc, const double* ptab,
                        int ntab, double w1, int B, int Hc, int Wc, void* stream);
int fea_transfer_weight_grad_f32(const float* cf, int c_split, const float* ff, int f_split, int C,
                                 int interior, float scale, float* gw, double* ws, int B, int Hc, int Wc,
                                 void* stream);
int fea_transfer_weight_grad_f64(const double* cf, int c_split, const double* ff, int f_split, int C,
                                 int interior, double scale, double* gw, double* ws, int B, int Hc, int Wc,
                                 void* stream);
/* Stencil-weight gradient of y = K u (and of conv3x3: ntab = 1, pid = NULL):
 *   gw[p][d] = scale * sum_i g[i] u[i+d] [pid(i+d) == p],  gw [ntab, 9]; ws holds
 *   fea_stencil_weight_grad_ws_bytes(ntab, B, H, W) bytes; fixed-order sums.  KNet / FNet / HNet
 *   weights (FEANet/model.py:22-30, 49-61; HNet M-FEANet-mg_test.ipynb:97-106). */
int fea_stencil_weight_grad_f32(const float* g, const float* u, const uint8_t* pid, int ntab, float scale,
                                float* gw, double* ws, int B, int H, int W, void* stream);
int fea_stencil_weight_grad_f64(const double* g, const double* u, const uint8_t* pid, int ntab, double scale,
                                double* gw, double* ws, int B, int H, int W, void* stream);
size_t fea_stencil_weight_grad_ws_bytes_f32(int ntab, int B, int H, int W);
size_t fea_stencil_weight_grad_ws_bytes_f64(int ntab, int B, int H, int W);
size_t fea_transfer_weight_grad_ws_bytes_f32(int C, int B, int Hc, int Wc);
size_t fea_transfer_weight_grad_ws_bytes_f64(int C, int B, int Hc, int Wc);

/* ---------------------------------------------------------------------------
 * (2) Framed multigrid-level ops (MultigridSolver), H x W grids (H, W >= 3; the intergrid ops need
 *     odd H and W: the coarse grid is (H+1)/2 x (W+1)/2, fine nodes (2I, 2J) on coarse (I, J)).
 *     `pid`/`pidc` are framed uint8 maps with the same ld (in bytes) as the T fields.
 *     Two-material stencils (ntab > 1): each node's stiffness weights are read from its own pattern's row with
 *     mirrored taps (ktab[p(i)][8-t] for tap t), which equals KNet's ktab[p(i+t)][t] (FEANet/model.py:22-30) bit for
 *     bit when K is a symmetric FE stiffness (stencil_table(); feanet_amd.mesh_setup.stencil_mirror_mismatches).
 * ------------------------------------------------------------------------- */

/* contiguous [B,1,H,W] -> framed, applying u*geo + bc (src NULL: u = 0; geo NULL: the square geometry,
 * or all ones if geo_bstride < 0 (a raw copy); bc NULL: zero) */
int fea_mg_pack_f32(const float* src, float* dst, const float* geo, long long geo_bstride,
                    const float* bc, long long bc_bstride, int B, int H, int W, int ld, long long bstride,
                    void* stream);
int fea_mg_pack_f64(const double* src, double* dst, const double* geo, long long geo_bstride,
                    const double* bc, long long bc_bstride, int B, int H, int W, int ld, long long bstride,
                    void* stream);
/* framed -> contiguous [B,1,H,W] */
int fea_mg_unpack_f32(const float* src, float* dst, int B, int H, int W, int ld, long long bstride, void* stream);
int fea_mg_unpack_f64(const double* src, double* dst, int B, int H, int W, int ld, long long bstride, void* stream);

/* Interior sweep out = J(u, f) (boundary untouched).  u == NULL: zero initial guess
 * (out = omd*f), the coarse-level pre-smooth of MultiGrid.iterate (FEANet/multigrid.py:171-172). */
int fea_mg_sweep_f32(const float* u, const float* f, float* out, const uint8_t* pid, const float* ktab,
                     const float* omd, int ntab, int B, int H, int W, int ld, long long bstride, void* stream);
int fea_mg_sweep_f64(const double* u, const double* f, double* out, const uint8_t* pid, const double* ktab,
                     const double* omd, int ntab, int B, int H, int W, int ld, long long bstride, void* stream);

/* Fused residual + restriction: fc(interior) = w0 * R(f - K u), kernel by fine-node pattern.
 * u == NULL: zero-initial-guess mode — the kernel first forms v = omd*f (the coarse-level
 * pre-smooth), writes it to v_out, and restricts f - K v (one read of f for three ops:
 * FEANet/multigrid.py:171-172 then :168-170).  v_out may be NULL: v is then not stored (the
 * prolongation recomputes it, fea_mg_prolong_sweep with u == NULL).  (ldc, bstridec) = coarse layout. */
int fea_mg_residual_restrict_f32(const float* u, const float* f, float* v_out, float* fc, const uint8_t* pid,
                                 const float* ktab, const float* omd, int ntab, const float* rtab, int nrtab,
                                 float w0, int B, int H, int W, int ld, long long bstride, int ldc,
                                 long long bstridec, void* stream);
int fea_mg_residual_restrict_f64(const double* u, const double* f, double* v_out, double* fc,
                                 const uint8_t* pid, const double* ktab, const double* omd, int ntab,
                                 const double* rtab, int nrtab, double w0, int B, int H, int W, int ld,
                                 long long bstride, int ldc, long long bstridec, void* stream);

/* Two zero-guess restrictions in one pass (the first two levels below the finest going down):
 *   v = omd*f;  fc = w0*R(f - K v);  v' = omd*fc;  fc2 = w0*R(fc - K v')     (interiors)
 * fc (the H_c x W_c level, pitch ldc / bstridec) is stored as well — the up pass recomputes v' from it —
 * and fc2 (pitch ldc2 / bstridec2) is the level below.  Bitwise the two fea_mg_residual_restrict calls
 * with u = v_out = NULL.  FEANet/multigrid.py:171-172 then :168-170 at two consecutive levels
 * (MultiGrid.Step's recursion, mg_test :27352-27363).  pidc: the coarse level's pattern map (ntab > 1). */
int fea_mg_zero_restrict2_f32(const float* f, float* fc, float* fc2, const uint8_t* pid, const uint8_t* pidc,
                              const float* ktab, const float* omd, int ntab, const float* rtab, int nrtab,
                              float w0, int B, int H, int W, int ld, long long bstride, int ldc,
                              long long bstridec, int ldc2, long long bstridec2, void* stream);
int fea_mg_zero_restrict2_f64(const double* f, double* fc, double* fc2, const uint8_t* pid, const uint8_t* pidc,
                              const double* ktab, const double* omd, int ntab, const double* rtab, int nrtab,
                              double w0, int B, int H, int W, int ld, long long bstride, int ldc,
                              long long bstridec, int ldc2, long long bstridec2, void* stream);

/* Domain-decomposed agglomeration (feanet_amd/dd.py; the restriction is FEANet/multigrid.py:168-172):
 * the zero-guess restrictions that produce the agglomerated level also store that level's block [r0, r1) x [c0, c1)
 * (local rows / columns of the output level) into send[b][r - r0][c - c0] — the all-gather's send buffer — so no copy
 * launch sits between the restriction and the all-gather.  Otherwise bitwise fea_mg_zero_restrict2 /
 * fea_mg_residual_restrict(u = v_out = NULL).  Nodes of the block outside the output level's interior are not
 * written (the caller keeps them zero). */
int fea_mg_zero_restrict2_send_f32(const float* f, float* fc, float* fc2, const uint8_t* pid, const uint8_t* pidc,
                                   const float* ktab, const float* omd, int ntab, const float* rtab, int nrtab,
                                   float w0, int B, int H, int W, int ld, long long bstride, int ldc,
                                   long long bstridec, int ldc2, long long bstridec2, float* send, int r0, int r1,
                                   int c0, int c1, void* stream);
int fea_mg_zero_restrict2_send_f64(const double* f, double* fc, double* fc2, const uint8_t* pid, const uint8_t* pidc,
                                   const double* ktab, const double* omd, int ntab, const double* rtab, int nrtab,
                                   double w0, int B, int H, int W, int ld, long long bstride, int ldc,
                                   long long bstridec, int ldc2, long long bstridec2, double* send, int r0, int r1,
                                   int c0, int c1, void* stream);
int fea_mg_zero_restrict_send_f32(const float* f, float* fc, const uint8_t* pid, const float* ktab, const float* omd,
                                  int ntab, const float* rtab, int nrtab, float w0, int B, int H, int W, int ld,
                                  long long bstride, int ldc, long long bstridec, float* send, int r0, int r1, int c0,
                                  int c1, void* stream);
int fea_mg_zero_restrict_send_f64(const double* f, double* fc, const uint8_t* pid, const double* ktab,
                                  const double* omd, int ntab, const double* rtab, int nrtab, double w0, int B, int H,
                                  int W, int ld, long long bstride, int ldc, long long bstridec, double* send, int r0,
                                  int r1, int c0, int c1, void* stream);

/* Fused pre-smooth + residual + restriction on a level with a given iterate (temporal blocking):
 *   u_out = J(u, f) (interior)   and   fc(interior) = w0 * R(f - K u_out)
 * u and f are read once.  FEANet/multigrid.py:165 then :168-170 (MultiGrid.Step, mg_test :27352-27357).
 * norm_hist != NULL: also the residual norm ||(f - K u)[b, 1:-1, 1:-1]||_2 of the INPUT iterate (the
 * drivers' initial residual, M-FEANet-mg_test.ipynb:27428-27429), appended to norm_hist as for
 * fea_mg_cycle_join below. */
int fea_mg_sweep_restrict_f32(const float* u, const float* f, float* u_out, float* fc, const uint8_t* pid,
                              const float* ktab, const float* omd, int ntab, const float* rtab, int nrtab,
                              float w0, int B, int H, int W, int ld, long long bstride, int ldc, long long bstridec,
                              double* norm_ws, double* norm_hist, unsigned* norm_cnt, void* stream);
int fea_mg_sweep_restrict_f64(const double* u, const double* f, double* u_out, double* fc, const uint8_t* pid,
                              const double* ktab, const double* omd, int ntab, const double* rtab, int nrtab,
                              double w0, int B, int H, int W, int ld, long long bstride, int ldc, long long bstridec,
                              double* norm_ws, double* norm_hist, unsigned* norm_cnt, void* stream);

/* Fused prolongation + correction + post-sweep:
 *   out = J(u + w1 * P(ec), f)   (P kernel by coarse-node pattern pidc)
 * FEANet/multigrid.py:177-181 (Interpolate, add, Relax) in one pass.
 * u == NULL: the level's iterate is its zero-guess pre-sweep omd*f (interior; 0 on the boundary),
 * recomputed from f — bitwise the v that fea_mg_residual_restrict(u = NULL) would have stored. */
int fea_mg_prolong_sweep_f32(const float* u, const float* ec, const float* f, float* out, const uint8_t* pid,
                             const uint8_t* pidc, const float* ktab, const float* omd, int ntab,
                             const float* ptab, int nptab, float w1, int B, int H, int W, int ld, long long bstride,
                             int ldc, long long bstridec, void* stream);
int fea_mg_prolong_sweep_f64(const double* u, const double* ec, const double* f, double* out,
                             const uint8_t* pid, const uint8_t* pidc, const double* ktab, const double* omd,
                             int ntab, const double* ptab, int nptab, double w1, int B, int H, int W, int ld,
                             long long bstride, int ldc, long long bstridec, void* stream);

/* Two recomputed-iterate prolongations + post-sweeps in one pass (the first two levels below the
 * multi-level launch going up):
 *   x' = omd*fc + w1*P(ec2);  u' = J(x', fc);  x = omd*f + w1*P(u');  out = J(x, f)     (interiors)
 * fc / pidc: the coarse level's right-hand side and pattern map (pitch ldc / bstridec), ec2 / pidc2: the
 * correction and pattern map of the level below it (pitch ldc2 / bstridec2).  u' is never stored.  Bitwise
 * fea_mg_prolong_sweep(u = NULL) on the coarse level, then on this one.  FEANet/multigrid.py:177-181 at two
 * consecutive levels (MultiGrid.Step's recursion unwinding, mg_test :27364-27372). */
int fea_mg_prolong2_f32(const float* fc, const float* ec2, const float* f, float* out, const uint8_t* pid,
                        const uint8_t* pidc, const uint8_t* pidc2, const float* ktab, const float* omd, int ntab,
                        const float* ptab, int nptab, float w1, int B, int H, int W, int ld, long long bstride,
                        int ldc, long long bstridec, int ldc2, long long bstridec2, void* stream);
int fea_mg_prolong2_f64(const double* fc, const double* ec2, const double* f, double* out, const uint8_t* pid,
                        const uint8_t* pidc, const uint8_t* pidc2, const double* ktab, const double* omd, int ntab,
                        const double* ptab, int nptab, double w1, int B, int H, int W, int ld, long long bstride,
                        int ldc, long long bstridec, int ldc2, long long bstridec2, void* stream);

/* Cycle join (temporal blocking across two V-cycles on one level): the post-smooth of cycle k and the
 * pre-smooth + residual + restriction of cycle k+1 in one pass —
 *   v = J(u + w1 * P(ec), f)  (not stored);   u_out = J(v, f);   fc(interior) = w0 * R(f - K u_out)
 * bitwise equal to fea_mg_prolong_sweep followed by fea_mg_sweep_restrict (FEANet/multigrid.py:177-181
 * then :165-170), reading u, f, ec once and writing u_out, fc (28 instead of 52 B per fp64 node).
 * norm_hist != NULL: also the drivers' residual norm of v, the end-of-cycle-k iterate
 * (||(f - K v)[b, 1:-1, 1:-1]||_2, M-FEANet-mg_test.ipynb:27428-27429), which the pre-smooth forms
 * anyway: appended as row norm_cnt[1] of norm_hist (B doubles per row; norm_cnt[1] += 1; norm_cnt[0]
 * unused), reduced deterministically by a one-workgroup kernel launched after the join on the same
 * stream; norm_ws >= fea_norm_workspace_bytes(B, H, W).  Replaces the per-cycle residual pass of the driver
 * loops (M-FEANet-mg_test.ipynb:27426-27436). */
int fea_mg_cycle_join_f32(const float* u, const float* ec, const float* f, float* u_out, float* fc,
                          const uint8_t* pid, const uint8_t* pidc, const float* ktab, const float* omd, int ntab,
                          const float* ptab, int nptab, const float* rtab, int nrtab, float w1, float w0, int B,
                          int H, int W, int ld, long long bstride, int ldc, long long bstridec, double* norm_ws,
                          double* norm_hist, unsigned* norm_cnt, void* stream);
int fea_mg_cycle_join_f64(const double* u, const double* ec, const double* f, double* u_out, double* fc,
                          const uint8_t* pid, const uint8_t* pidc, const double* ktab, const double* omd, int ntab,
                          const double* ptab, int nptab, const double* rtab, int nrtab, double w1, double w0, int B,
                          int H, int W, int ld, long long bstride, int ldc, long long bstridec, double* norm_ws,
                          double* norm_hist, unsigned* norm_cnt, void* stream);

/* Prolongation + correction without a sweep (nu2 = 0 schedules): out = u + w1 * P(ec), interior. */
int fea_mg_prolong_add_f32(const float* u, const float* ec, float* out, const uint8_t* pidc, const float* ptab,
                           int nptab, float w1, int B, int H, int W, int ld, long long bstride, int ldc,
                           long long bstridec, void* stream);
int fea_mg_prolong_add_f64(const double* u, const double* ec, double* out, const uint8_t* pidc,
                           const double* ptab, int nptab, double w1, int B, int H, int W, int ld, long long bstride,
                           int ldc, long long bstridec, void* stream);

/* The cycle join (fea_mg_cycle_join, no residual norm) over nrect <= 4 rectangles of the grid in one launch:
 * rects[4 r ..] = {I0, I1, c0, c1}: coarse rows [I0, I1) (their fine rows 2I-1, 2I; row H-2 with I1 = Hc-1) and
 * fine columns [c0, c1), c0 odd, c1 odd or W-1 (coarse column J with fine columns 2J-1, 2J).  Rectangles covering the
 * grid give fea_mg_cycle_join's result bitwise; a domain-decomposed rank computes the border strips its halo
 * exchange sends first and the interior while the messages are in flight (feanet_amd.dd). */
int fea_mg_cycle_join_rects_f32(const float* u, const float* ec, const float* f, float* u_out, float* fc,
                                const uint8_t* pid, const uint8_t* pidc, const float* ktab, const float* omd, int ntab,
                                const float* ptab, int nptab, const float* rtab, int nrtab, float w1, float w0, int B,
                                int H, int W, int ld, long long bstride, int ldc, long long bstridec, int nrect,
                                const int* rects, void* stream);
int fea_mg_cycle_join_rects_f64(const double* u, const double* ec, const double* f, double* u_out, double* fc,
                                const uint8_t* pid, const uint8_t* pidc, const double* ktab, const double* omd,
                                int ntab, const double* ptab, int nptab, const double* rtab, int nrtab, double w1,
                                double w0, int B, int H, int W, int ld, long long bstride, int ldc, long long bstridec,
                                int nrect, const int* rects, void* stream);

/* out[b] = || (f - K u)[b, rlo:rhi, 1:-1] ||_2 (rows rlo..rhi-1; rlo = rhi = 0: all interior rows,
 * the drivers' [1:-1, 1:-1]; likewise columns clo..chi-1, clo = chi = 0: all interior columns),
 * deterministic; ws >= fea_norm_workspace_bytes(B, H, W).  Row and column ranges give a
 * domain-decomposed rank the sum over the nodes it owns. */
int fea_mg_residual_norm_f32(const float* u, const float* f, const uint8_t* pid, const float* ktab, int ntab,
                             double* out, double* ws, int B, int H, int W, int ld, long long bstride, int rlo,
                             int rhi, int clo, int chi, void* stream);
int fea_mg_residual_norm_f64(const double* u, const double* f, const uint8_t* pid, const double* ktab, int ntab,
                             double* out, double* ws, int B, int H, int W, int ld, long long bstride, int rlo,
                             int rhi, int clo, int chi, void* stream);

/* One sweep of the learned smoother (HJacIterator.HRelax, M-FEANet-mg_test.ipynb:147-155, HNet
 * :97-106) fused in one pass:  j = J(u, f);  d = (W_nl * .. (W_1 * (j - u)) .g ..) .g;  out = j + d
 * on the interior (boundary untouched).  hw = nlayers 3x3 conv weights (cross-correlation, zero
 * padding; nlayers <= 3), g = interior mask.  u == NULL: zero initial guess (coarse levels).
 * u_raw (optional, framed like u): the iterate as the caller passed it before reset_boundary — the
 * reference forms j - u with the un-reset u, so a first sweep from a guess whose boundary is not the
 * Dirichlet data sees (bc - u_raw) on the boundary nodes; NULL = u already holds the boundary. */
int fea_mg_hsweep_f32(const float* u, const float* u_raw, const float* f, float* out, const uint8_t* pid,
                      const float* ktab, const float* omd, int ntab, const float* hw, int nlayers, int B, int H,
                      int W, int ld, long long bstride, void* stream);
int fea_mg_hsweep_f64(const double* u, const double* u_raw, const double* f, double* out, const uint8_t* pid,
                      const double* ktab, const double* omd, int ntab, const double* hw, int nlayers, int B,
                      int H, int W, int ld, long long bstride, void* stream);
/* The learned smoother fused with the inter-grid transfers around it (the streamed MG-HJac level pair of
 * M-FEANet-mg_test.ipynb MultiGrid.Step :27346-27372, one pass each instead of two):
 * hsweep_restrict: out = HRelax(u) as fea_mg_hsweep (u NULL: zero guess; u_raw as there), then
 *   fc = w0 R(f - K out) on the (H+1)/2 x (W+1)/2 level (framed ldc, bsc) as fea_mg_residual_restrict with a
 *   stored iterate.  prolong_hsweep: x = u + w1 P(ec) on the interior (fea_mg_prolong_add, ec = the coarse
 *   correction), then out = HRelax(x); u_raw as for fea_mg_hsweep (the first sweep of a cycle after a load with
 *   no pre-sweep sees the un-reset guess on the boundary).  Both bitwise the two launches they replace; H, W odd; out != u. */
int fea_mg_hsweep_restrict_f32(const float* u, const float* u_raw, const float* f, float* out, float* fc,
                               const uint8_t* pid, const float* ktab, const float* omd, int ntab, const float* hw,
                               int nlayers, const float* rtab, int nrtab, float w0, int B, int H, int W, int ld,
                               long long bstride, int ldc, long long bstridec, void* stream);
int fea_mg_hsweep_restrict_f64(const double* u, const double* u_raw, const double* f, double* out, double* fc,
                               const uint8_t* pid, const double* ktab, const double* omd, int ntab, const double* hw,
                               int nlayers, const double* rtab, int nrtab, double w0, int B, int H, int W, int ld,
                               long long bstride, int ldc, long long bstridec, void* stream);
int fea_mg_prolong_hsweep_f32(const float* u, const float* u_raw, const float* ec, const float* f, float* out,
                              const uint8_t* pid,
                              const uint8_t* pidc, const float* ktab, const float* omd, int ntab, const float* hw,
                              int nlayers, const float* ptab, int nptab, float w1, int B, int H, int W, int ld,
                              long long bstride, int ldc, long long bstridec, void* stream);
int fea_mg_prolong_hsweep_f64(const double* u, const double* u_raw, const double* ec, const double* f, double* out,
                              const uint8_t* pid,
                              const uint8_t* pidc, const double* ktab, const double* omd, int ntab, const double* hw,
                              int nlayers, const double* ptab, int nptab, double w1, int B, int H, int W, int ld,
                              long long bstride, int ldc, long long bstridec, void* stream);

/* The whole coarse end of the V-cycle (levels t..t+nlev-1 of an Ht x Wt level, Ht, Wt <= 65 and
 * (Ht-1), (Wt-1) divisible by 2^(nlev-1)) in ONE launch,
 * one 1024-thread workgroup per sample, every level resident in LDS.  Input f_t and output v_t
 * are framed level-t buffers (ld_t, bs_t); v_t's interior is written.  The sub-cycle starts from a
 * zero guess: nu1 pre-sweeps per level (none if q2), nu1+nu2 (q2: nu2) sweeps on the coarsest,
 * prolongation + correction + nu2 post-sweeps (FEANet/multigrid.py:165-183 below level t).
 * pid_levels: the nlev compact H_k x W_k uint8 pattern maps concatenated (NULL when ntab == 1);
 * rtab/ptab hold ntab kernels (broadcast single kernels on the host). */
int fea_mg_coarse_tail_f32(const float* f_t, float* v_t, int Ht, int Wt, int nlev, int ld_t, long long bs_t,
                           const uint8_t* pid_levels, const float* ktab, const float* omd, int ntab,
                           const float* rtab, const float* ptab, float w0, float w1, int nu1, int nu2, int q2,
                           int B, void* stream);
int fea_mg_coarse_tail_f64(const double* f_t, double* v_t, int Ht, int Wt, int nlev, int ld_t, long long bs_t,
                           const uint8_t* pid_levels, const double* ktab, const double* omd, int ntab,
                           const double* rtab, const double* ptab, double w0, double w1, int nu1, int nu2,
                           int q2, int B, void* stream);
/* The coarse tail with the level above it (level X: Hx = 2 Ht - 1 rows, Wx = 2 Wt - 1 <= 129 columns, framed f_x /
 * v_x with ld_x, bs_x) in the same launch: X's zero-guess restriction (fea_mg_residual_restrict with u = NULL and no
 * iterate stored) into the tail's LDS, the tail's nlev levels, then X's recomputed-iterate prolongation + sweep
 * (fea_mg_prolong_sweep with u = NULL) into v_x's interior — bitwise those three launches
 * (FEANet/multigrid.py:165-183 for the levels below the one above X).  Single pattern (ntab == 1), V(1,1). */
int fea_mg_coarse_tail_ext_f32(const float* f_x, float* v_x, int Hx, int Wx, int ld_x, long long bs_x, int nlev,
                               const float* ktab, const float* omd, int ntab, const float* rtab, const float* ptab,
                               float w0, float w1, int B, void* stream);
int fea_mg_coarse_tail_ext_f64(const double* f_x, double* v_x, int Hx, int Wx, int ld_x, long long bs_x, int nlev,
                               const double* ktab, const double* omd, int ntab, const double* rtab,
                               const double* ptab, double w0, double w1, int B, void* stream);
/* LDS bytes the coarse tail needs for (Ht, Wt, nlev); 0 if unsupported.  Must be <= 159 KiB. */
size_t fea_mg_coarse_tail_lds_bytes(int Ht, int Wt, int nlev, int elem_size, int multi);

/* The coarse end of the learned-smoother V-cycle (MultiGrid.Step mode='hjac', M-FEANet-mg_test.ipynb:27346-27372
 * with Relax = HJacIterator.HRelax :147-155) for levels t..t+nlev-1 of an Ht x Wt level (Ht, Wt <= 65) in ONE
 * launch, one 1024-thread workgroup per sample, every level resident in LDS (hjac_tail.hip).  From a zero guess:
 * nu1 HRelax pre-sweeps per level, residual + restriction, nu1+nu2 sweeps on the coarsest, prolongation +
 * correction + nu2 post-sweeps; hw = nlayers 3x3 HNet weights.  Bitwise the per-level fea_mg_hsweep /
 * fea_mg_residual_restrict / fea_mg_prolong_add sequence it replaces (feanet_amd.schedule.hjac_schedule).
 * f_t / u_t: framed level-t buffers (ld_t, bs_t); u_t's interior is written.  pid_levels as for the coarse tail. */
int fea_mg_hjac_tail_f32(const float* f_t, float* u_t, int Ht, int Wt, int nlev, int ld_t, long long bs_t,
                         const uint8_t* pid_levels, const float* ktab, const float* omd, int ntab, const float* rtab,
                         const float* ptab, const float* hw, int nlayers, float w0, float w1, int nu1, int nu2, int B,
                         void* stream);
int fea_mg_hjac_tail_f64(const double* f_t, double* u_t, int Ht, int Wt, int nlev, int ld_t, long long bs_t,
                         const uint8_t* pid_levels, const double* ktab, const double* omd, int ntab,
                         const double* rtab, const double* ptab, const double* hw, int nlayers, double w0, double w1,
                         int nu1, int nu2, int B, void* stream);
/* LDS bytes the learned-smoother tail needs for (Ht, Wt, nlev); 0 if unsupported.  Must be <= 159 KiB. */
size_t fea_mg_hjac_tail_lds_bytes(int Ht, int Wt, int nlev, int elem_size, int multi);

/* Several consecutive coarse levels in ONE launch (mid_ops.hip; tiles with recomputed halos, bitwise
 * the per-level kernels).  Levels a .. a+k (k <= 4) are framed buffers (fea_mg_layout) of H x W,
 * (H+1)/2 x (W+1)/2, ...; pid[j] their pattern maps (NULL array when ntab == 1).
 * mid_down: the zero-guess pre-sweep + residual + restriction of levels a .. a+k-1 (V(1,1) down leg,
 *   FEANet/multigrid.py:171-172 then :168-170, one fea_mg_residual_restrict(u = NULL) per level):
 *   reads f[0] = f_a, writes f[1..k] = f_{a+1} .. f_{a+k} (interior).  Tile TR x TC of level a+k.
 * mid_up: the prolongation + correction + post-sweep of levels a+k-1 .. a from e = u_{a+k}
 *   (:177-181, one fea_mg_prolong_sweep(u = NULL) per level): reads f[0..k-1] = f_a .. f_{a+k-1},
 *   writes out = u_a (interior); intermediate iterates are not stored.  Tile TR x TC of level a.
 * Both return FEA_EINVAL if the tile's LDS footprint (fea_mg_mid_lds_bytes) does not fit. */
int fea_mg_mid_down_f32(const float* const* f, const uint8_t* const* pid, int k, int B, int H, int W,
                        const float* ktab, const float* omd, int ntab, const float* rtab, int nrtab, float w0,
                        int TR, int TC, void* stream);
int fea_mg_mid_down_f64(const double* const* f, const uint8_t* const* pid, int k, int B, int H, int W,
                        const double* ktab, const double* omd, int ntab, const double* rtab, int nrtab, double w0,
                        int TR, int TC, void* stream);
/* mid_down of the agglomerated coarse problem of a domain-decomposed run (feanet_amd/dd.py): level a's f is read
 * from the all-gather's buffer gsrc ([Pr * Pc][B][gcr][gcc], rank r's block of gcr x gcc nodes starting at
 * node (1 + (r / Pc) gcr, 1 + (r % Pc) gcc); H - 1 = Pr gcr, W - 1 = Pc gcc) instead of f[0], and every tile also
 * writes the interior nodes it owns into f[0] (framed) for the later launches — the placement copy of the
 * gathered blocks folded into this launch.  Otherwise bitwise fea_mg_mid_down on the placed f[0]. */
int fea_mg_mid_down_gathered_f32(const float* const* f, const uint8_t* const* pid, int k, int B, int H, int W,
                                 const float* ktab, const float* omd, int ntab, const float* rtab, int nrtab, float w0,
                                 int TR, int TC, const float* gsrc, int Pr, int Pc, int gcr, int gcc, void* stream);
int fea_mg_mid_down_gathered_f64(const double* const* f, const uint8_t* const* pid, int k, int B, int H, int W,
                                 const double* ktab, const double* omd, int ntab, const double* rtab, int nrtab,
                                 double w0, int TR, int TC, const double* gsrc, int Pr, int Pc, int gcr, int gcc,
                                 void* stream);
int fea_mg_mid_up_f32(const float* const* f, const float* e, float* out, const uint8_t* const* pid, int k, int B,
                      int H, int W, const float* ktab, const float* omd, int ntab, const float* ptab, int nptab,
                      float w1, int TR, int TC, void* stream);
int fea_mg_mid_up_f64(const double* const* f, const double* e, double* out, const uint8_t* const* pid, int k,
                      int B, int H, int W, const double* ktab, const double* omd, int ntab, const double* ptab,
                      int nptab, double w1, int TR, int TC, void* stream);
/* LDS bytes of one mid launch (up = 0 down, 1 up) with a full TR x TC tile; -1 if it does not fit. */
long long fea_mg_mid_lds_bytes(int up, int k, int TR, int TC, int elem_size, int multi);

/* Two consecutive coarse levels a, a+1 of the learned-smoother V(1,1) cycle in ONE launch each way (hmid_ops.hip;
 * tiles with recomputed halos, every stage an LDS pass; bitwise the streaming kernels they replace).  Levels a,
 * a+1, a+2 are framed buffers (fea_mg_layout) of H x W, (H+1)/2 x (W+1)/2, ...; pid[0..2] their pattern maps
 * (NULL array when ntab == 1); hw = nlayers 3x3 HNet weights.
 * hmid_down: the zero-guess HRelax pre-sweep + residual + restriction of levels a and a+1 (two
 *   fea_mg_hsweep_restrict(u = NULL) calls, M-FEANet-mg_test.ipynb MultiGrid.Step :27346-27360 with
 *   Relax = HJacIterator.HRelax :147-155): reads f[0] = f_a, writes u[0] = u_a, f[1] = f_(a+1), u[1] = u_(a+1),
 *   f[2] = f_(a+2) (interior).  Tile T x T of level a+2.
 * hmid_up: the prolongation + correction + HRelax post-sweep of levels a+1 and a from e = u_(a+2) (two
 *   fea_mg_prolong_hsweep calls, :27362-27372): reads f[0..1] = f_a, f_(a+1), u[0..1] = the stored iterates
 *   u_a, u_(a+1); writes out = the new u_a (interior); the new u_(a+1) is not stored.  Tile T x T of level a.
 * Both return FEA_EINVAL if the tile's LDS footprint (fea_mg_hmid_lds_bytes) does not fit. */
int fea_mg_hmid_down_f32(const float* const* f, float* const* u, const uint8_t* const* pid, int B, int H, int W,
                         const float* ktab, const float* omd, int ntab, const float* hw, int nlayers,
                         const float* rtab, int nrtab, float w0, int T, void* stream);
int fea_mg_hmid_down_f64(const double* const* f, double* const* u, const uint8_t* const* pid, int B, int H, int W,
                         const double* ktab, const double* omd, int ntab, const double* hw, int nlayers,
                         const double* rtab, int nrtab, double w0, int T, void* stream);
int fea_mg_hmid_up_f32(const float* const* f, const float* const* u, const float* e, float* out,
                       const uint8_t* const* pid, int B, int H, int W, const float* ktab, const float* omd, int ntab,
                       const float* hw, int nlayers, const float* ptab, int nptab, float w1, int T, void* stream);
int fea_mg_hmid_up_f64(const double* const* f, const double* const* u, const double* e, double* out,
                       const uint8_t* const* pid, int B, int H, int W, const double* ktab, const double* omd,
                       int ntab, const double* hw, int nlayers, const double* ptab, int nptab, double w1, int T,
                       void* stream);
/* LDS bytes of one hmid launch (up = 0 down, 1 up) with a full T x T tile; -1 if it does not fit. */
long long fea_mg_hmid_lds_bytes(int up, int T, int nlayers, int elem_size, int multi);

/* Domain decomposition (feanet_amd.dd): the halo exchange's pack / unpack in one launch.
 * blocks: HOST array of nblocks records {int64 frame (device address of a block in a framed buffer),
 * int64 stage (device address of the block in a staging buffer), int64 ld (row pitch, elements), int32 rows,
 * int32 cols}, copied into the kernel arguments (48 blocks per launch); to_stage = 1 copies every block into
 * its stage (row-major, rows x cols), 0 back out of it.  elem_size 4 or 8.  No reference counterpart (the
 * reference is single-process): it packs the messages of the new multi-GPU path. */
int fea_dd_copy_blocks(const void* blocks, int nblocks, int elem_size, int to_stage, void* stream);
/* Strided rectangle copies in one launch (the agglomeration's all-gather staging / placement and the coarse
 * solution's scatter, feanet_amd.dd): rects is a HOST array of nrects records {int64 dst, int64 src (device
 * addresses of the first elements), int64 dst_ld, int64 src_ld (row pitches, elements), int64 rows, int64 cols},
 * copied into the kernel arguments (32 per launch).  elem_size 4 or 8.  No reference counterpart. */
int fea_dd_copy_rects(const void* rects, int nrects, int elem_size, void* stream);

/* On-device mesh set-up: the MeshCenterInterface node pattern map — replaces
 * FEANet/mesh.py place_circle / place_rect (:62-76), identify_patterns (:78-93) and
 * generate_global_pattern_map (:95-101) with one thread per node, bit-identical to the reference's
 * float32 geometry.  out[r * ld + c] = pattern id (0..15) of node (r, c), 0 on the boundary;
 * shape 0 = circle, 1 = square inclusion; size = plate edge length (the reference's `size`). */
int fea_interface_pattern_map(uint8_t* out, long long ld, int N, int shape, double size, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FEANET_HIP_H */
