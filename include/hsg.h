/*
 * hsg.h -- C ABI of the MI355X-native WSWGAT hot path (libhsg.so, gfx950).
 *
 * The reference (yellow-binary-tree/HeterSumGraph) has no FFI: its hot path is the
 * Python operator WSWGAT(...).forward(g, w, s) (module/GAT.py:31-59) built from DGL
 * UDFs (module/GATLayer.py:81-152) and a per-head Python loop
 * (module/GATStackLayer.py:55-63).  Each entry point below replaces one piece of
 * that call chain; the Python host layer (hetersumgraph_amd/module/) binds them
 * with ctypes exactly as shown in INTEGRATION.md.
 *
 * Conventions
 *   - All pointers are device pointers (hipMalloc'd or torch-allocated).  The
 *     library never allocates, frees or synchronises; work is enqueued on `stream`
 *     (a hipStream_t passed as void*), so every call is graph-capturable.
 *   - Row-major fp32 features.  Z is [n_src, H*D], head k occupies columns
 *     [k*D, (k+1)*D) (the torch.cat order of GATStackLayer.py:59).
 *   - Return value: 0 on success, otherwise a hipError_t (launch error) or
 *     HSG_EINVAL for unsupported shapes.  No global mutable state; reentrant
 *     across streams and devices.
 */
#ifndef HSG_H_
#define HSG_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HSG_EINVAL 1001

/* One typed relation (W2S: word->sentence/doc, S2W: sentence/doc->word).
 * Replaces, per layer call, DGL's filter_nodes/filter_edges
 * (GATLayer.py:105-107, 143-145) and the in-edge set of g.pull (113, 149). */
typedef struct hsg_rel {
    int32_t n_src;            /* |source set|      (rows of Z, sigma)               */
    int32_t n_dst;            /* |destination set| (rows of the output)             */
    int32_t n_edges;          /* |typed edges| E_T                                  */
    const int32_t *indptr;    /* [n_dst+1] CSR by destination rank                  */
    const int32_t *src;       /* [E_T]     source rank per CSR edge                 */
    const uint8_t *tf;        /* [E_T]     tau row per CSR edge (tf-idf box, 10=0)  */
    const int32_t *phantom;   /* [n_dst]   untyped in-edges (e=0, z=0) per dst      */
    const int32_t *cindptr;   /* [n_src+1] CSC by source rank                       */
    const int32_t *cdst;      /* [E_T]     destination rank per CSC edge            */
    const int32_t *cperm;     /* [E_T]     CSR position of each CSC edge            */
    /* Work lists for degree-skewed relations (round 6; hsg_rel_work): 0 / NULL = none.
     * Items in node order, [n][4] = (node, beg, end, first): node >= 0 is a whole node,
     * node = -(v + 1) one piece [beg, end) of a long segment of node v (the HDSG doc
     * supernodes' ~250 word edges, dataloader.py:387-400, next to ~20 per sentence),
     * first = the item index of v's first piece; then [n] arrival counters (zero, or a
     * multiple of v's piece count at the first piece's slot, between launches).  dwork
     * splits the CSR (destinations: hsg_gat_fwd_ws), swork the CSC (sources:
     * hsg_gat_bwd_src_g_ws); the pieces' partial results are merged in a fixed order.
     * The counters make launches that use one work list stream-ordered: do not run
     * two such launches on one relation concurrently. */
    int32_t n_dwork;          /* items of dwork (0: no CSR work list)               */
    int32_t n_swork;          /* items of swork (0: no CSC work list)               */
    int32_t *dwork;           /* [n_dwork][4] items + [n_dwork] counters             */
    int32_t *swork;           /* [n_swork][4] items + [n_swork] counters             */
} hsg_rel;

/* tau addressing: HSG_TAU_TABLE -> tau is [11, H] indexed by rel->tf (tf-idf box
 * table, HiGraph.py:52 + zero row); HSG_TAU_PER_EDGE -> tau is [E_T, H] in CSR order
 * (a foreign caller wrote a dense edata['tfidfembed']). */
#define HSG_TAU_TABLE 0
#define HSG_TAU_PER_EDGE 1

/* Forward of one multi-head WSGAT/SWGAT application, all heads fused.
 * Replaces GATLayer.py:89-93 (edge_attention, apply_edges), 95-102
 * (message_func/reduce_func under g.pull with degree bucketing), the head loop and
 * concat of GATStackLayer.py:55-59 and -- when `origin` != NULL -- the ELU +
 * residual of GAT.py:56-57:
 *   s_e   = leaky_relu(sigma[src_e,k] + tau[t_e,k], slope)
 *   m_v   = max(max_e s_e, 0 if phantom_v>0),  l_v = sum_e exp(s_e-m_v) + phantom_v*exp(-m_v)
 *   h[v]  = sum_e exp(s_e-m_v)/l_v * Z[src_e, k, :]      (0 if v has no in-edges)
 *   out   = origin ? elu(h) + origin : h
 * Saved for backward: h, m, l ([n_dst, H] each).  With an origin, h may be NULL (not
 * stored): the backward is then hsg_gat_bwd_dst_noh. */
int hsg_gat_fwd(const hsg_rel *rel, int H, int D, int tau_mode, float slope,
                const float *Z, const float *sigma, const float *tau, const float *origin,
                float *h, float *out, float *m, float *l, void *stream);
/* hsg_gat_fwd with the relation's CSR work list (round 6): a destination whose typed
 * in-edges exceed the list's piece length is aggregated as pieces -- (max, sum, partial
 * h) per piece written to ws, then merged with its phantoms in piece order by a second
 * launch (the same online-softmax algebra; deterministic).  ws holds
 * hsg_gat_fwd_ws_floats(rel, H, D) floats (0: no work list, ws may be NULL and the call
 * equals hsg_gat_fwd).  Multi-wave (long-segment) forward only; other shapes ignore the
 * list. */
size_t hsg_gat_fwd_ws_floats(const hsg_rel *rel, int H, int D);
int hsg_gat_fwd_ws(const hsg_rel *rel, int H, int D, int tau_mode, float slope, const float *Z,
                   const float *sigma, const float *tau, const float *origin, float *h, float *out, float *m,
                   float *l, float *ws, void *stream);
/* hsg_gat_fwd_ws with an origin, the result x = elu(h) + origin stored as bf16 rows
 * (round-to-nearest-even) of pitch ld16 in out16 INSTEAD of the fp32 out (out may be
 * NULL): the bf16 GEMM mode's bf16 x rows (round 6) -- the wide FFN's A operand,
 * LayerNorm residual and dW1 operand.  ld16 % 8 == 0, ld16 >= ceil8(H*D), out16 16-byte
 * aligned; columns H*D .. ld16 - 1 are written zero (the bf16-A contract of
 * hsg_gemm_bf16_psw_io).  Per element |x16 - x| <= 2^-9 |x|. */
int hsg_gat_fwd_ws16(const hsg_rel *rel, int H, int D, int tau_mode, float slope, const float *Z,
                     const float *sigma, const float *tau, const float *origin, float *h, float *out, float *m,
                     float *l, float *ws, void *out16, int ld16, void *stream);

/* Backward, destination-centric half: given dOut, computes
 *   G = origin_mode ? dOut * elu'(h) : dOut                      [n_dst, H*D]
 *   dpre[e,k] = alpha_ek (G_v.Z_u - G_v.h_v) * leaky'(pre_ek)   [E_T, H], CSR order
 *   dtau_part[b, t, k] = per-block partial sums of dpre by tau row (table mode)
 * dtau_part must hold hsg_gat_bwd_blocks(rel) * 11 * H floats. */
int hsg_gat_bwd_dst(const hsg_rel *rel, int H, int D, int tau_mode, int origin_mode, float slope,
                    const float *Z, const float *sigma, const float *tau,
                    const float *h, const float *m, const float *l, const float *dout,
                    float *G, float *dpre, float *dtau_part, void *stream);

/* Number of partial rows hsg_gat_bwd_dst writes into dtau_part. */
int hsg_gat_bwd_blocks(const hsg_rel *rel);

/* hsg_gat_bwd_dst with origin_mode = 1 for a forward that did not store h
 * (hsg_gat_fwd with h = NULL): elu'(h) from x - origin (x = the forward's out) and
 * G_v.h_v = sum_e alpha_ek G_v.Z_u over the typed edges.  Same outputs and dtau_part
 * rows as hsg_gat_bwd_dst; hsg_gat_bwd_dst_noh_supported(rel, H, D) tells whether the
 * shape has this form (the feature-split pass: D > 16, short segments). */
int hsg_gat_bwd_dst_noh_supported(const hsg_rel *rel, int H, int D);
int hsg_gat_bwd_dst_noh(const hsg_rel *rel, int H, int D, int tau_mode, float slope,
                        const float *Z, const float *sigma, const float *tau,
                        const float *x, const float *origin, const float *m, const float *l,
                        const float *dout, float *G, float *dpre, float *dtau_part, void *stream);

/* hsg_gat_bwd_dst_noh with the G rows given (origin_mode 1, e.g. from
 * hsg_gemm_f32_psw_elug): G is read, not written; dpre and dtau_part as
 * hsg_gat_bwd_dst.  Supported where hsg_gat_bwd_dst_noh_supported. */
int hsg_gat_bwd_dst_g(const hsg_rel *rel, int H, int D, int tau_mode, float slope,
                      const float *Z, const float *sigma, const float *tau, const float *m, const float *l,
                      const float *G, float *dpre, float *dtau_part, void *stream);

/* Backward, source-centric half (CSC): for every source u
 *   dZ[u, k, :]  = sum_{e: src_e = u} alpha_ek * G[dst_e, k, :]  (+ dsigma[u,k]*a1[k,:] if a1)
 *   dsigma[u, k] = sum_{e: src_e = u} dpre[e, k]                 (written if dsigma != NULL)
 *   da1_part[b, k*D+d] = per-block partial sums of dsigma[u,k] * Z[u,k,d]
 *                  (if da1_part != NULL; needs Z and hsg_gat_bwd_src_blocks(rel)*H*D floats)
 * a1 (optional, [H, D]) folds the gradient of sigma = <Z[u,k,:], a1[k,:]> into dZ. */
int hsg_gat_bwd_src(const hsg_rel *rel, int H, int D, int tau_mode, float slope,
                    const float *sigma, const float *tau, const float *m, const float *l,
                    const float *G, const float *dpre, const float *a1, const float *Z,
                    float *dZ, float *dsigma, float *da1_part, void *stream);

/* Number of partial rows hsg_gat_bwd_src writes into da1_part. */
int hsg_gat_bwd_src_blocks(const hsg_rel *rel);

/* The whole backward of one table-mode application in ONE source-centric pass (the
 * S2W shape: D in [32, 64], long CSC segments -- hsg_gat_bwd_src_g_supported), given
 * G = dOut * elu'(h) and rho[v][g][s] = the per-64-column-group partials of
 * G_v . h_v that hsg_gemm_psw_elug_rho writes (rho_groups = ceil(H*D / W), W its group width):
 *   dpre[e,k]   = alpha_ek (G[v,k,:] . Z[u,k,:] - rho_vk) * leaky'(pre_ek)
 *   dZ, dsigma, da1_part as hsg_gat_bwd_src, dtau_part[b][box][k] per-block partials
 * with b < hsg_gat_bwd_src_g_blocks(rel, H, D) for both slabs.  Replaces hsg_gat_bwd_dst_g +
 * hsg_gat_bwd_src (GATLayer.py:118-131 backward); results equal up to fp32 rounding
 * (rho is summed from G.h instead of sum_e alpha_e G.Z_u). */
/* rho_groups == 0: the narrow-head shape (D = 8, H <= 8, short CSC segments: the W2S
 * words) with rho[v][k] = G_v,k . h_v,k per head, as hsg_ffn_small_bwd_gate writes it
 * (the head-lane kernel; G, Z, dZ, a1 16-byte aligned). */
int hsg_gat_bwd_src_g_supported(const hsg_rel *rel, int H, int D);
/* Number of partial rows hsg_gat_bwd_src_g writes into da1_part and dtau_part. */
int hsg_gat_bwd_src_g_blocks(const hsg_rel *rel, int H, int D);
int hsg_gat_bwd_src_g(const hsg_rel *rel, int H, int D, float slope, const float *sigma, const float *tau,
                      const float *m, const float *l, const float *G, const float *rho, int rho_groups,
                      const float *a1, const float *Z, float *dZ, float *dsigma, float *da1_part,
                      float *dtau_part, void *stream);
/* hsg_gat_bwd_src_g with G as bf16 rows when g_bf16 != 0 (the bf16 GEMM mode: the G
 * hsg_gemm_bf16_psw_elug_rho_a16 writes with g_bf16; wide heads only, rho_groups > 0). */
int hsg_gat_bwd_src_g_io(const hsg_rel *rel, int H, int D, float slope, const float *sigma, const float *tau,
                         const float *m, const float *l, const void *G, int g_bf16, const float *rho, int rho_groups,
                         const float *a1, const float *Z, float *dZ, float *dsigma, float *da1_part,
                         float *dtau_part, void *stream);
/* hsg_gat_bwd_src_g_io with the relation's CSC work list (round 6): a source whose
 * out-edges exceed the piece length is walked as pieces (one block each), their dZ
 * and dsigma partials written to ws and summed in piece order by a second launch, which
 * adds dsigma * a1 (da1 / dtau partials stay per block).  ws holds
 * hsg_gat_bwd_src_g_ws_floats(rel, H, D) floats (0: no work list; the call equals
 * hsg_gat_bwd_src_g_io).  Wide heads only; the narrow head-lane kernel ignores the list. */
size_t hsg_gat_bwd_src_g_ws_floats(const hsg_rel *rel, int H, int D);
int hsg_gat_bwd_src_g_ws(const hsg_rel *rel, int H, int D, float slope, const float *sigma, const float *tau,
                         const float *m, const float *l, const void *G, int g_bf16, const float *rho, int rho_groups,
                         const float *a1, const float *Z, float *dZ, float *dsigma, float *da1_part,
                         float *dtau_part, float *ws, void *stream);

/* Measurement hook (bench.py's in-step kernel clock; not part of the reference
 * surface): the next hsg_gat_fwd launched FROM THE CALLING THREAD ON `stream` records
 * start_event / stop_event (hipEvent_t created with timing) from its kernel's own
 * dispatch packet (hipExtLaunchKernel); the next hsg_gat_bwd_dst records start_event
 * at its kernel and the following hsg_gat_bwd_src stop_event at its kernel.  One-shot:
 * a consumed event is disarmed.  Either event may be NULL (disarm).  The armed state
 * is thread-local and bound to `stream`, so launches from other threads or onto other
 * streams are unaffected.  hsg_kclock_pending: bit 0 / bit 1 set while the calling
 * thread's start / stop is still armed. */
int hsg_kclock_arm(void *stream, void *start_event, void *stop_event);
int hsg_kclock_pending(void);

/* sigma[u, k] = <Z[u, k, :], a1[k, :]> -- the z_src part of attn_fc
 * (GATLayer.py:91-92 / 130-131); a1 = attn_fc.weight[0, :D] per head. */
int hsg_attn_src_logits(int n, int H, int D, const float *Z, const float *a1, float *sigma,
                        void *stream);

/* ---- attention parameters of one layer application (GATLayer.py:84-93, 123-131) ----
 * attn [H][3D] = the heads' attn_fc weights [a1 | a2 | a3] (a2 multiplies the
 * all-zero z_dst, GATLayer.py:111), wf [H][D][F] / bf [H][D] (NULL on W2S) the
 * feat_fc weights, T [10][F] the TF-IDF embedding table (HiGraph.py:52).
 * fwd: a1 [H][D] = attn[:, :D];  tau [11][H]: tau[t][k] = <a3_k, wf_k T[t] + bf_k>
 *      for t < 10, tau[10][k] = <a3_k, bf_k> (edges whose tfidfembed stayed 0).
 * bwd: reduces dtau_part (hsg_gat_bwd_dst, n_dtau_part rows of 11*H) and da1_part
 *      (hsg_gat_bwd_src, n_da1_part rows of H*D) in a fixed order (two launches,
 *      hsg_attn_params_bwd_workspace_floats(H, D) floats of workspace) and writes
 *      dattn [H][3D] (= [da1 | 0 | da3]), dwf [H][D][F], dbf [H][D] (if bf and dbf),
 *      dT [10][F] -- or adds into those buffers (a layer applied several times
 *      per step: the gradient sums over its applications): accumulate bit 0 for
 *      dattn / dwf / dbf, bit 1 for dT (the table is shared by both layer kinds).
 *      H <= 16, H*D <= 512, F <= 256. */
int hsg_attn_params_fwd(int H, int D, int F, const float *attn, const float *wf, const float *bf,
                        const float *T, float *a1, float *tau, void *stream);

/* The attention tables of TWO layers sharing the TF-IDF table T (the fused stack's
 * W2S and S2W, once per forward) in one launch: for each layer exactly what
 * hsg_attn_params_fwd writes (a1 [H, D], tau [11, H]).  Replaces the two per-layer
 * launches of the same GATLayer.py:84-93 / 123-131 edge-type term. */
int hsg_attn_params_fwd_pair(int H0, int D0, const float *attn0, const float *wf0, const float *bf0, float *a1_0,
                             float *tau0, int H1, int D1, const float *attn1, const float *wf1, const float *bf1,
                             float *a1_1, float *tau1, int F, const float *T, void *stream);
/* hsg_attn_params_fwd_pair that also performs the step's dropout-seed advance in the
 * same launch (seed[0] += 1; snap[0] = the new value: hsg_seed_advance), so the fused
 * stack's forward starts with one launch instead of two.  seed and snap both given or
 * both NULL (then exactly hsg_attn_params_fwd_pair).  Nothing else may read seed or
 * snap before this launch completes (stream order). */
int hsg_attn_params_fwd_pair_seed(int H0, int D0, const float *attn0, const float *wf0, const float *bf0,
                                  float *a1_0, float *tau0, int H1, int D1, const float *attn1, const float *wf1,
                                  const float *bf1, float *a1_1, float *tau1, int F, const float *T, int64_t *seed,
                                  int64_t *snap, void *stream);
int hsg_attn_params_bwd(int H, int D, int F, int n_dtau_part, const float *dtau_part, int n_da1_part,
                        const float *da1_part, const float *attn, const float *wf, const float *bf,
                        const float *T, float *dattn, float *dwf, float *dbf, float *dT, float *workspace,
                        int accumulate, void *stream);
/* The same backward in its two stages, so several applications of one layer can
 * share the parameter transform: hsg_attn_params_stage reduces one application's
 * partial slabs into the workspace (accumulate != 0: added to what the workspace
 * holds -- the slabs of earlier applications of the same layer, in call order);
 * hsg_attn_params_finish turns the accumulated workspace into the parameter
 * gradients (accumulate flags as hsg_attn_params_bwd).  The transform is linear,
 * so stage(a1) + stage(a2) -> finish equals finish(a1) + finish(a2) up to fp32
 * summation order. */
int hsg_attn_params_stage(int H, int D, int n_dtau_part, const float *dtau_part, int n_da1_part,
                          const float *da1_part, float *workspace, int accumulate, void *stream);
int hsg_attn_params_finish(int H, int D, int F, const float *workspace, const float *attn, const float *wf,
                           const float *bf, const float *T, float *dattn, float *dwf, float *dbf, float *dT,
                           int accumulate, void *stream);

/* hsg_attn_params_finish of two layers sharing T (the fused stack's W2S and S2W) in
 * one launch: the same gradients, and when both layers name the same dT, layer 0's
 * update of each element is applied before layer 1's, exactly as two launches in
 * that order (acc0 / acc1: the accumulate flags of the two calls). */
int hsg_attn_params_finish_pair(int H0, int D0, const float *ws0, const float *attn0, const float *wf0,
                                const float *bf0, float *dattn0, float *dwf0, float *dbf0, float *dT0, int acc0,
                                int H1, int D1, const float *ws1, const float *attn1, const float *wf1,
                                const float *bf1, float *dattn1, float *dwf1, float *dbf1, float *dT1, int acc1,
                                int F, const float *T, void *stream);
size_t hsg_attn_params_bwd_workspace_floats(int H, int D);

/* ---- dense fp32 GEMM on the matrix cores ---------------------------------------
 * Replaces the torch GEMMs of the head projection fc (GATLayer.py:110 / 146) and of
 * PositionwiseFeedForward (Conv1d k=1 = GEMM, GATLayer.py:39) plus their backward.
 * hsg_gemm_f32: fp32 operands and result, fp32-accurate products computed as six
 * bf16 limb products per element pair (each operand split into three bf16 limbs when
 * its tile is staged; v_mfma_f32_32x32x16_bf16, fp32 accumulation; dropped terms
 * <= ~3*2^-24 |a b|, the error class of an fp32 fmaf chain).
 * hsg_gemm_f32_mfma: same contract on the exact-f32 instruction v_mfma_f32_32x32x2_f32
 * (one fmaf rounding per product; 2.67x lower MFMA ceiling).
 *   C[m][n] = epi( sum_k A(m,k) B(k,n) )
 *   A(m,k) = a_kcontig ? A[m*lda+k] : A[k*lda+m];  B(k,n) = b_kcontig ? B[n*ldb+k] : B[k*ldb+n]
 * epi: HSG_EPI_STORE    v (+bias[n]) then relu if `relu`
 *      HSG_EPI_RELU_BWD v * (aux[m][n] > 0)
 *      HSG_EPI_ADD      v (+bias[n]) + aux[m][n]     (aux may alias C: accumulate)
 * splits > 1: split-K over `splits` slices; needs hsg_gemm_workspace_floats() floats
 * of workspace; the slices are reduced in order (deterministic).  splits == 0:
 * choose automatically (split only when the output has too few tiles).
 * Requires lda, ldb multiples of 4 and 16-byte aligned A, B. */
#define HSG_EPI_STORE 0
#define HSG_EPI_RELU_BWD 1
#define HSG_EPI_ADD 2
#define HSG_EPI_ADD_ELUG 3   /* hsg_gemm_f32_psw_elug only */
size_t hsg_gemm_workspace_floats(int M, int N, int K, int splits);   /* splits 0: the automatic plan */
int hsg_gemm_auto_splits(int M, int N, int K);
int hsg_gemm_f32(int M, int N, int K, const float *A, int lda, int a_kcontig,
                 const float *B, int ldb, int b_kcontig, float *C, int ldc,
                 const float *bias, const float *aux, int ldaux, int epi, int relu,
                 int splits, float *workspace, float *colsum_part, void *stream);
/* colsum_part (optional, unsplit GEMMs only): per-tile-row column sums of the stored
 * C, [hsg_gemm_row_tiles(M,N,K,splits)][N] -- e.g. the bias gradient of the FFN's
 * first layer taken from the dH epilogue instead of a second pass over dH. */
int hsg_gemm_row_tiles(int M, int N, int K, int splits);
int hsg_gemm_f32_mfma(int M, int N, int K, const float *A, int lda, int a_kcontig,
                      const float *B, int ldb, int b_kcontig, float *C, int ldc,
                      const float *bias, const float *aux, int ldaux, int epi, int relu,
                      int splits, float *workspace, float *colsum_part, void *stream);
/* Pre-split weights (the FFN's W1, W2 and their transposes, SURVEY §8a step 4:
 * reference module/PositionwiseFeedForward.py:23-34 w_1/w_2).  hsg_wsplit writes, for
 * each of njobs (1..4) weights, the three bf16 limb planes of the [N][K] matrix
 * B = trans ? W^T : W (W row pitch ldw floats) into planes[q] = bf16 [3][Np][Kp]
 * (hsg_wsplit_dims: Np = N rounded up to 128, Kp = K rounded up to 32, zero padded),
 * limbs as hsg_gemm_f32's split.  hsg_gemm_f32_psw is hsg_gemm_f32 for
 * C = A B^T with a K-contiguous fp32 A (K % 4 == 0) and B given by its planes: the
 * weight is split once per step instead of once per row tile of every GEMM.  Same
 * epilogues and colsum_part rows (hsg_gemm_row_tiles) as hsg_gemm_f32, no split-K. */
void hsg_wsplit_dims(int N, int K, int *Np, int *Kp);
int hsg_wsplit(int njobs, const float *const *W, const int *N, const int *K, const int *ldw,
               const int *trans, void *const *planes, void *stream);
int hsg_gemm_f32_psw(int M, int N, int K, const float *A, int lda, const void *planes,
                     float *C, int ldc, const float *bias, const float *aux, int ldaux,
                     int epi, int relu, float *colsum_part, void *stream);
/* The FFN backward's last GEMM with the edge layer's ELU gate fused into its epilogue
 * (GAT.py:56-57 backward; replaces the dOut -> G step of hsg_gat_bwd_dst):
 *   C = aux + A B^T          (dx = ds + dH W1: the FFN input's gradient, = the origin's)
 *   G = C * elu'(h),  elu'(h) = 1 if e > 0 else e + 1,  e = x - origin = elu(h)
 * x: the edge layer's output (the FFN input), origin: its residual input; aux, x,
 * origin and G share the row pitch `ld`.  N % 4 == 0 and 16-byte aligned rows
 * (HSG_EINVAL otherwise: the caller keeps the split path).  The G rows feed
 * hsg_gat_bwd_dst_g. */
int hsg_gemm_f32_psw_elug(int M, int N, int K, const float *A, int lda, const void *planes, float *C, int ldc,
                          const float *aux, const float *x, const float *origin, float *G, int ld, int bf16,
                          void *stream);
/* hsg_gemm_f32_psw_elug that also writes rho (optional: NULL = the call above) for
 * hsg_gat_bwd_src_g: rho[m][g][s], g < ceil(N / W), s < 3, = sum of G[m,c] * h[m,c]
 * over the columns c of group g (Wg <= c < Wg + W) in head c / head_dim =
 * Wg / head_dim + s, h = e for e > 0 else log1p(e); head_dim >= 32 divides N.  The
 * group width W = hsg_gemm_psw_elug_rho_gw(M, N, K, head_dim, bf16): 64, or 112 in the
 * fp32 mode for N <= 320 (the GEMM's 112-wide tiles; round 5) when every group meets at
 * most three heads. */
int hsg_gemm_psw_elug_rho(int M, int N, int K, const float *A, int lda, const void *planes, float *C, int ldc,
                          const float *aux, const float *x, const float *origin, float *G, int ld, float *rho,
                          int head_dim, int bf16, void *stream);
int hsg_gemm_psw_elug_rho_gw(int M, int N, int K, int head_dim, int bf16);
/* hsg_gemm_bf16 (A and the weight rounded to bf16 RNE, fp32 accumulation: config 5's
 * mode) on the pre-split weight: only its limb plane 0 = RNE(W) is read, one bf16
 * MFMA product per element pair.  Same arguments as hsg_gemm_f32_psw; N % 4 == 0 and
 * 16-byte aligned C / aux rows (HSG_EINVAL otherwise).  hsg_gemm_f32_psw_elug with
 * bf16 != 0 has these numerics too. */
int hsg_gemm_bf16_psw(int M, int N, int K, const float *A, int lda, const void *planes, float *C, int ldc,
                      const float *bias, const float *aux, int ldaux, int epi, int relu, float *colsum_part,
                      void *stream);
/* The bf16 mode's FFN GEMMs on bf16 activations (round 5): hsg_gemm_bf16_psw with A,
 * C and the relu' mask aux given as bf16 rows per io = HSG_IO_A_BF16 | HSG_IO_C_BF16 |
 * HSG_IO_AUX_BF16 (io in {0, 1, 2, 3, 7}; element strides lda / ldc / ldaux).  A bf16 A
 * needs lda % 8 == 0, 16-byte alignment and zeros in its columns K .. ceil8(K) - 1; a
 * bf16 C takes no accumulate epilogue, a bf16 aux only the relu' mask.  The bf16 mode
 * rounds A to bf16 at fragment read anyway, so the products equal hsg_gemm_bf16_psw's on
 * the same values; a bf16 C is the fp32 result rounded to nearest even. */
#define HSG_IO_A_BF16 1
#define HSG_IO_C_BF16 2
#define HSG_IO_AUX_BF16 4
int hsg_gemm_bf16_psw_io(int M, int N, int K, const void *A, int lda, const void *planes, void *C, int ldc,
                         const float *bias, const void *aux, int ldaux, int epi, int relu, float *colsum_part,
                         int io, void *stream);
/* hsg_gemm_psw_elug_rho in the bf16 mode with a bf16 A (the FFN's bf16 dH rows; the
 * bf16 A contract above); g_bf16: G stored as bf16 rows (pitch ld; rho is summed from
 * the fp32 G), for hsg_gat_bwd_src_g_io. */
int hsg_gemm_bf16_psw_elug_rho_a16(int M, int N, int K, const void *A, int lda, const void *planes, float *C,
                                   int ldc, const float *aux, const float *x, const float *origin, void *G, int ld,
                                   float *rho, int head_dim, int g_bf16, void *stream);
/* ... with x given as bf16 rows of pitch ldx when x_bf16 != 0 (hsg_gat_fwd_ws16's rows;
 * ldx % 8 == 0; G must be bf16 then, g_bf16 != 0): elu(h) = x - origin from the bf16 x.
 * x_bf16 == 0: hsg_gemm_bf16_psw_elug_rho_a16 (x fp32, pitch ld). */
int hsg_gemm_bf16_psw_elug_rho_x16(int M, int N, int K, const void *A, int lda, const void *planes, float *C,
                                   int ldc, const float *aux, const void *x, int ldx, int x_bf16, const float *origin,
                                   void *G, int ld, float *rho, int head_dim, int g_bf16, void *stream);
/* Same contract as hsg_gemm_f32 (fp32 A, B, C, epilogues, split-K, colsum_part), but
 * the MFMA takes A and B rounded to bf16 (round-to-nearest-even) and accumulates in
 * fp32 (v_mfma_f32_32x32x16_bf16): the reduced-precision mode of config 5 (NYT50,
 * bf16).  Products of bf16 values are exact in fp32, so the result equals
 * an fp32 GEMM of the rounded operands up to fp32 summation order. */
/* hsg_gemm_f32's split-K pass alone: workspace[splits][M][N] receives the K-slice
 * products, summed by hsg_slab_reduce (splits >= 2). */
int hsg_gemm_f32_slabs(int M, int N, int K, const float *A, int lda, int a_kcontig,
                       const float *B, int ldb, int b_kcontig, int splits, float *workspace,
                       void *stream);
/* The same for hsg_gemm_bf16 (operands rounded to bf16 RNE, one product). */
int hsg_gemm_bf16_slabs(int M, int N, int K, const float *A, int lda, int a_kcontig,
                        const float *B, int ldb, int b_kcontig, int splits, float *workspace,
                        void *stream);
/* The S2W FFN's second GEMM with dropout + residual + LayerNorm in its epilogue
 * (GATLayer.py:39-42: y = w_2(relu(...)) + b2, out = LayerNorm(dropout(y) + x)):
 * y = A B^T + bias (pre-split B, hsg_wsplit planes; bf16 != 0: the bf16 mode's one
 * product), out, mean, rstd exactly as hsg_ln_fwd on that y (same dropout stream:
 * seed[0], offset, index r*N + c).  y, x, out contiguous [M][N].  HSG_EINVAL when the
 * shape has no one-round full-row plan (N <= 320, 60-100 % of the CUs busy): the caller
 * then runs hsg_gemm_*_psw + hsg_ln_fwd. */
int hsg_gemm_psw_ln(int M, int N, int K, const float *A, int lda, const void *planes, const float *bias, float *y,
                    const float *x, const float *gamma, const float *beta, float eps, float p_drop, const int64_t *seed,
                    uint32_t offset, float *out, float *mean, float *rstd, int bf16, void *stream);
/* Rows of the column-partial slab (colsum_part [rows][N]) hsg_gemm_f32_psw /
 * hsg_gemm_bf16_psw write for an M x N x K GEMM: the big-tile plan of the cfg2-class
 * shapes sums per 80- / 48-row band, the others per 64 rows (hsg_gemm_row_tiles). */
int hsg_gemm_psw_row_tiles(int M, int N, int K, int bf16);
/* The FFN weight gradients of one layer in ONE launch (replaces PositionwiseFeedForward's
 * dW2 = dY^T H and dW1 = dH^T X backward, module/GATLayer.py:39-41, summed over every
 * application's rows): job q (njobs 1..2) computes the split-K partial products of
 * A_q^T B_q with A_q [K][M_q] (row stride lda_q) and B_q [K][N_q] (ldb_q), both
 * M/N-contiguous, into ws_q[splits][M_q][N_q], summed later by hsg_slab_reduce.
 * fp32-accurate (three bf16 limbs per operand, six products), or with bf16 != 0 the
 * bf16 mode's one product of RNE-rounded operands.  Requires M, N, lda, ldb multiples
 * of 4 and 16-byte aligned A, B (HSG_EINVAL otherwise); splits must leave every K
 * slice non-empty (ceil(ceil(K/32) / ceil(ceil(K/32)/splits)) == splits). */
int hsg_gemm_dw_slabs(int njobs, const int *M, const int *N, int K, const float *const *A, const int *lda,
                      const float *const *B, const int *ldb, int splits, int bf16, float *const *ws, void *stream);
/* hsg_gemm_dw_slabs in the bf16 mode with bf16 operands (round 5): io[q] bit 0 -- A_q is
 * bf16 rows, bit 1 -- B_q is bf16 rows (element strides; 8-byte quads, M / N / ld
 * multiples of 4, 16-byte aligned).  The products equal the bf16 mode's on the same
 * values. */
int hsg_gemm_dw_slabs_io(int njobs, const int *M, const int *N, int K, const void *const *A, const int *lda,
                         const void *const *B, const int *ldb, const int *io, int splits, float *const *ws,
                         void *stream);
/* Output tiles of one hsg_gemm_dw_slabs job of shape M x N (blocks = tiles x splits). */
int hsg_gemm_dw_tiles(int M, int N);
/* Deferred column sums of partial slabs, njobs (1..24) outputs in one deterministic
 * launch: out[q][b][c] = (accumulate[q] ? out[q][b][c] : 0) + scale[q] * sum over
 * job q's nseg[q] (1..4) segments s (in order) of the rows r in the b-th of
 * out_rows[q] equal row ranges of s of seg_s[r*pitch[q] + coff[q] + c], c < cols[q]
 * (out_rows 1: plain column sums; > 1: a staged partial [out_rows][cols], e.g. the
 * hsg_attn_params_stage workspace).  seg / seg_rows list the segments of all jobs
 * back to back.  The fused stack's backward sums every layer's head-projection dW
 * slabs, FFN bias / LayerNorm partials, attention-parameter partials and split-K
 * weight gradients here, once per step, instead of one launch per application. */
int hsg_slab_reduce(int njobs, float *const *out, const int *cols, const int *out_rows, const int *pitch,
                    const int *coff, const float *scale, const int *accumulate, const int *nseg,
                    const float *const *seg, const int *seg_rows, void *stream);
int hsg_gemm_bf16(int M, int N, int K, const float *A, int lda, int a_kcontig,
                  const float *B, int ldb, int b_kcontig, float *C, int ldc,
                  const float *bias, const float *aux, int ldaux, int epi, int relu,
                  int splits, float *workspace, float *colsum_part, void *stream);

/* ---- PositionwiseFeedForward row epilogue (GATLayer.py:40-42) -------------------
 * Forward:  s = dropout(y; p, seed, offset) + x;  out = (s-mean)*rstd*gamma + beta
 *           (y = W2 relu(W1 x + b1) + b2 from hsg_gemm_f32; eps as nn.LayerNorm)
 * Backward: dx = dLN/ds (residual branch), dy = dx * mask / (1-p),
 *           part[b][3][d] = per-block column partials of dgamma, dbeta and dy
 *           (= the bias gradient of W2); hsg_ln_bwd_blocks(n) blocks, sum in order.
 * Dropout masks are a stateless hash of (*seed, offset, element index): *seed is
 * read from device memory (advance it between graph replays), offset is a
 * per-call constant; forward and backward with equal (seed, offset) agree.
 * d <= 512; p_drop in [0, 1). */
int hsg_ln_bwd_blocks(int n);
/* The FFN backward's bias / LayerNorm parameter gradients, one launch, fixed order:
 *   db1[c] = sum_r hpart[r][c]                        (hsg_gemm_f32 colsum_part of dH)
 *   dgamma[c], dbeta[c], db2[c] = sum_r lnpart[r][0..2][c]      (hsg_ln_bwd part)
 * accumulate != 0: add into the outputs (a layer applied several times per step). */
int hsg_ffn_colsums(int rows_h, int d_hid, const float *hpart, float *db1, int rows_ln, int d,
                    const float *lnpart, float *dgamma, float *dbeta, float *db2, int accumulate,
                    void *stream);
/* The whole FFN forward in one launch for the narrow W2S FFN (d = 64, d_hid = 512;
 * hsg_ffn_small_supported(d, d_hid) says whether a shape is covered):
 *   H = relu(x W1^T + b1) [n][d_hid],  y = H W2^T + b2 [n][d],
 *   out = LN(dropout(y) + x) with mean / rstd -- the outputs of hsg_gemm_f32 x 2 +
 *   hsg_ln_fwd (same dropout hash and index, so hsg_ln_bwd takes y, mean, rstd).
 * w1 [d_hid][d], w2 [d][d_hid] row-major; x, w1, w2 16-byte aligned. */
int hsg_ffn_small_supported(int d, int d_hid);
int hsg_ffn_small_fwd(int n, int d, int d_hid, const float *x, const float *w1, const float *b1,
                      const float *w2, const float *b2, const float *gamma, const float *beta, float eps,
                      float p_drop, const int64_t *seed, uint32_t offset, float *H, float *y, float *out,
                      float *mean, float *rstd, void *stream);
/* Its backward up to the weight gradients, one launch (hsg_ln_bwd + the dH and dx
 * GEMMs of the split path):  dy = LN/dropout backward of dout, dH = (dy W2) * (H > 0),
 * dx = dLN/ds + dH W1;  lnpart [blocks][3][d] (dgamma, dbeta, db2 partials) and
 * hpart [blocks][d_hid] (db1 partials) for hsg_ffn_colsums, blocks =
 * hsg_ffn_small_bwd_blocks(n).  dW1 = dH^T x and dW2 = dy^T H stay hsg_gemm_f32. */
int hsg_ffn_small_bwd_blocks(int n);
int hsg_ffn_small_bwd(int n, int d, int d_hid, const float *dout, const float *x, const float *H,
                      const float *y, const float *w1, const float *w2, const float *gamma,
                      const float *mean, const float *rstd, float p_drop, const int64_t *seed,
                      uint32_t offset, float *dy, float *dH, float *dx, float *lnpart, float *hpart,
                      void *stream);
/* hsg_ffn_small_bwd that also hands the W2S edge layer its backward operands from dx
 * (= the edge layer's dOut; GAT.py:56-57, GATLayer.py:118-131): G = dx * elu'(h)
 * (1 for h > 0, else exp(h)) and rho[row][k] = sum over head k's 8 columns of G * h,
 * h_edge the edge layer's saved h [n][d] (d = 64 = 8 heads x 8), for
 * hsg_gat_bwd_src_g with rho_groups = 0.  HSG_EINVAL when a pointer is NULL. */
int hsg_ffn_small_bwd_gate(int n, int d, int d_hid, const float *dout, const float *x, const float *H,
                           const float *y, const float *w1, const float *w2, const float *gamma, const float *mean,
                           const float *rstd, float p_drop, const int64_t *seed, uint32_t offset, float *dy,
                           float *dH, float *dx, float *lnpart, float *hpart, const float *h_edge, float *G,
                           float *rho, void *stream);
int hsg_ln_fwd(int n, int d, const float *y, const float *x, const float *gamma, const float *beta,
               float eps, float p_drop, const int64_t *seed, uint32_t offset,
               float *out, float *mean, float *rstd, void *stream);
int hsg_ln_bwd(int n, int d, const float *dout, const float *y, const float *x, const float *gamma,
               const float *mean, const float *rstd, float p_drop, const int64_t *seed, uint32_t offset,
               float *dy, float *dx, float *part, void *stream);
/* hsg_ln_bwd with dy stored as bf16 rows of pitch ld_dy (the bf16 GEMM mode, where dy is
 * only a GEMM operand; y_bf16: y read as bf16 rows of pitch d, as hsg_ln_fwd_y16
 * wrote it): zeros in its columns d .. ceil8(d) - 1; the vector kernel's
 * shapes only (d % 4 == 0, 257..512 columns, 16-byte aligned rows, ld_dy % 8 == 0),
 * HSG_EINVAL otherwise.  dx and the partials as hsg_ln_bwd (db2 sums the fp32 dy). */
int hsg_ln_bwd_dy16(int n, int d, const float *dout, const void *y, int y_bf16, const float *x, const float *gamma,
                    const float *mean, const float *rstd, float p_drop, const int64_t *seed, uint32_t offset,
                    void *dy, int ld_dy, float *dx, float *part, void *stream);
/* hsg_ln_fwd with the FFN output y given as bf16 rows of pitch d (the bf16 GEMM mode:
 * y is the GEMM's fp32 result rounded to nearest even, per-row error <= 2^-9 |y|); the
 * persistent vector kernel's shapes only (d % 4 == 0, 257..512 columns), HSG_EINVAL
 * otherwise.  hsg_ln_bwd_dy16 takes the same y with y_bf16 != 0. */
int hsg_ln_fwd_y16(int n, int d, const void *y, const float *x, const float *gamma, const float *beta, float eps,
                   float p_drop, const int64_t *seed, uint32_t offset, float *out, float *mean, float *rstd,
                   void *stream);
/* hsg_ln_fwd_y16 / hsg_ln_bwd_dy16 (bf16 y, pitch d; bf16 dy rows of pitch ld_dy) with the
 * residual x also given as bf16 rows, pitch ldx (% 8 == 0, >= ceil8(d), 16-byte aligned):
 * hsg_gat_fwd_ws16's rows (round 6).  out, mean, rstd, dx and the partials as hsg_ln_fwd /
 * hsg_ln_bwd on the bf16 values of y and x; HSG_EINVAL off the vector kernels' shapes. */
int hsg_ln_fwd_x16(int n, int d, const void *y, const void *x, int ldx, const float *gamma, const float *beta,
                   float eps, float p_drop, const int64_t *seed, uint32_t offset, float *out, float *mean, float *rstd,
                   void *stream);
int hsg_ln_bwd_x16(int n, int d, const float *dout, const void *y, const void *x, int ldx, const float *gamma,
                   const float *mean, const float *rstd, float p_drop, const int64_t *seed, uint32_t offset, void *dy,
                   int ld_dy, float *dx, float *part, void *stream);

/* ---- head projection with per-head input dropout (GATStackLayer.py:56) ----------
 * Training-mode  z_k = fc_k(dropout_k(h))  for all heads without materialising the
 * H dropped copies of h (reference: GATLayer.py:110 / :146 apply nn.Dropout to the
 * layer input inside each head's forward):
 *   hsg_dropmask: keep(i, k, c) as bits, a stateless hash of (*seed, offset, i, k, c)
 *                 with 16-bit resolution in p; layout, NWI = ceil(n/32),
 *                 LDC = in rounded up to 4:
 *                   bits[(k*NWI + i/32)*LDC + c] bit (i%32)
 *                 hsg_dropmask_words(n,in,H) uint32 words.
 *   hsg_hproj_fwd: Z[i, kD+d]  = s * sum_c bit X[i,c] W[kD+d, c]
 *   hsg_hproj_dx:  dX[i, c]    = s * sum_k bit sum_d dZ[i, kD+d] W[kD+d, c]
 *   hsg_hproj_dw:  dW[kD+d, c] = s * sum_i dZ[i, kD+d] bit X[i,c]
 *                  (part: hsg_hproj_dw_chunks(n,in,H,D) * H*D*in floats of workspace)
 * W is the fused fc weight [H*D][in] (row-major); s = 1/(1-p_eff) =
 * hsg_dropmask_scale(p).  Any H, D >= 1.  dx / dw with accumulate != 0 add into
 * dX / dW instead of overwriting them. */
int hsg_dropmask_words(int n, int in, int H);
float hsg_dropmask_scale(float p);
int hsg_dropmask(int n, int in, int H, float p, const int64_t *seed, uint32_t offset, uint32_t *bits,
                 void *stream);
/* One-launch seed step of the dropout stream (rng.DropoutRNG.advance): seed[0] += 1 and
 * snap[0] = the new seed (the snapshot the step's forward and backward share). */
int hsg_seed_advance(int64_t *seed, int64_t *snap, void *stream);
/* njobs (1..8) masks in one launch, job q identical to
 * hsg_dropmask(n[q], in[q], H[q], p[q], seed, offset[q], bits[q]): the fused stack draws
 * the masks of all its head projections up front. */
int hsg_dropmask_multi(int njobs, const int *n, const int *in, const int *H, const float *p,
                       const int64_t *seed, const uint32_t *offset, uint32_t *const *bits, void *stream);

/* hsg_dropmask_multi plus, in the same launch, the narrow-head projection's weight
 * transpose Wt[k][c][d] = W[k*wD+d][c] of hsg_hproj_wt (H = wH, D = wD, in = wIn;
 * W == NULL: masks only).  Both depend on the step's seed / the parameters only,
 * so the fused stack draws its keep-masks and transposes W2S's weight in one
 * launch (GATStackLayer.py:56 dropout, GATLayer.py:110 fc). */
int hsg_dropmask_multi_wt(int njobs, const int *n, const int *in, const int *H, const float *p,
                          const int64_t *seed, const uint32_t *offset, uint32_t *const *bits, int wH, int wD,
                          int wIn, const float *W, float *Wt, void *stream);

/* The step's parameter-only prologue in ONE launch: hsg_dropmask_multi_wt's masks and
 * weight transpose, plus hsg_wsplit's limb planes of nsplit (0..4) weights (sW, sN,
 * sK, sldw, strans, splanes as hsg_wsplit's W, N, K, ldw, trans, planes): the fused
 * stack's dropout masks (GATStackLayer.py:56), W2S fc weight (GATLayer.py:110) and
 * the S2W FFN's w_1 / w_2 views (GATLayer.py:39), all independent of the step's
 * activations. */
int hsg_step_prologue(int njobs, const int *n, const int *in, const int *H, const float *p, const int64_t *seed,
                      const uint32_t *offset, uint32_t *const *bits, int wH, int wD, int wIn, const float *W,
                      float *Wt, int nsplit, const float *const *sW, const int *sN, const int *sK, const int *sldw,
                      const int *strans, void *const *splanes, void *stream);
int hsg_hproj_fwd(int n, int in, int H, int D, const float *X, int ldx, const float *W,
                  const uint32_t *bits, float p, float *Z, int ldz, void *stream);
/* hsg_hproj_fwd plus the attention's source logits sigma[i][k] = <Z[i, kD:(k+1)D], a1[k]>
 * (a1 [H][D]; sigma [n][H]) from the same launch -- hsg_attn_src_logits fused into the
 * projection's epilogue.  hsg_hproj_fwd_logits_supported(H, D): whether the fused form
 * covers (H, D) (ceil(D/16) divides 4); a1 = sigma = NULL is hsg_hproj_fwd. */
int hsg_hproj_fwd_logits_supported(int H, int D);
int hsg_hproj_fwd_logits(int n, int in, int H, int D, const float *X, int ldx, const float *W,
                         const uint32_t *bits, float p, float *Z, int ldz, const float *a1, float *sigma,
                         void *stream);
/* Narrow heads (D = 8: the W2S projection, GATStackLayer.py:56 with 8 heads x 8) on
 * the f32 VALU: hsg_hproj_fwd_logits with the weight given transposed per head,
 * Wt[k][c][d] = W[kD+d][c] (hsg_hproj_wt, once per forward; H*in*8 floats).  Same
 * Z, sigma and keep bits.  hsg_hproj_fwd_t8_supported(in, H, D): D == 8, in % 4 == 0;
 * X and Z 16-byte aligned with ldx, ldz multiples of 4. */
int hsg_hproj_wt(int H, int D, int in, const float *W, float *Wt, void *stream);
int hsg_hproj_fwd_t8_supported(int in, int H, int D);
int hsg_hproj_fwd_t8(int n, int in, int H, const float *X, int ldx, const float *Wt, const uint32_t *bits,
                     float p, float *Z, int ldz, const float *a1, float *sigma, void *stream);
/* The D = 8 forward on bf16 limb MFMAs (round 5): the same Z / sigma as
 * hsg_hproj_fwd_t8 to fp32 rounding, W given as its hsg_wsplit limb planes
 * [3][Np][Kp] (hsg_wsplit_dims(H*8, in)).  H <= 8, in % 4 == 0, X 16-byte aligned. */
int hsg_hproj_fwd_mf_supported(int in, int H, int D);
int hsg_hproj_fwd_mf(int n, int in, int H, const float *X, int ldx, const void *planes, int Np, int Kp,
                     const uint32_t *bits, float p, float *Z, int ldz, const float *a1, float *sigma, void *stream);
int hsg_hproj_dx(int n, int in, int H, int D, const float *dZ, int ldz, const float *W,
                 const uint32_t *bits, float p, float *dX, int ldx, int accumulate, void *stream);
/* dX and the dW partial slabs of one projection (hsg_hproj_dx + hsg_hproj_dw with
 * dW = NULL: part holds hsg_hproj_dw_chunks(n, in, H, D) slabs [H*D][in], unscaled)
 * in ONE launch where both would be small wide-head launches (the S2W shape: heads
 * of D <= 64, few rows), else the two launches.  X row pitch ldx, dX row pitch ldxo. */
int hsg_hproj_bwd(int n, int in, int H, int D, const float *dZ, int ldz, const float *W, const float *X, int ldx,
                  const uint32_t *bits, float p, float *dX, int ldxo, int accumulate, float *part, void *stream);
int hsg_hproj_dw_chunks(int n, int in, int H, int D);
/* dW == NULL: only the partial slabs part[chunk][H*D][in] (unscaled), to be summed
 * with scale hsg_dropmask_scale(p) by hsg_slab_reduce. */
int hsg_hproj_dw(int n, int in, int H, int D, const float *dZ, int ldz, const float *X, int ldx,
                 const uint32_t *bits, float p, float *part, float *dW, int accumulate, void *stream);

/* Device construction of one typed relation from the batched graph's COO edges.
 * Replaces DGL's per-call filter_nodes/filter_edges (GATLayer.py:105-107, 143-145),
 * the in-edge set of g.pull (113, 149) and the tffrac -> _TFembed row selection of
 * HSumGraph.set_wnfeature (HiGraph.py:146-151); runs once per batch.
 *   src, dst   [E] int64 node ids;  unit [n] float (dataloader.py:216-217, 0 word / 1 sentence|doc)
 *   tffrac     [E] int64 (nullable -> tau row 10 everywhere); edtype [E] float (nullable -> all 0)
 * Sources are nodes with unit == src_unit, destinations unit == dst_unit, typed edges
 * go source -> destination.  Outputs are sized by the upper bounds n and E; the true
 * sizes land in counts[0..2] = n_src, n_dst, n_typed (device).  counts[3] = typed
 * dtype-0 edges whose tffrac is outside the 10 boxes (nn.Embedding would raise),
 * counts[4] = edges with a node id outside [0, n): the caller raises on either.
 *   indptr [n+1] (first n_dst+1 valid), esrc/tf/eid [E] (first n_typed), phantom [n],
 *   cindptr [n+1] (first n_src+1), cdst/cperm [E], src_nodes/dst_nodes [n] int64.
 * CSR edges of one destination keep edge-id order (the DGL mailbox order); CSC edges of
 * one source keep CSR order.  workspace >= hsg_rel_build_workspace_bytes(n, E). */
/* Work list of one CSR / CSC (round 6, hsg_rel.dwork / swork): with mean segment m =
 * indptr[n] / n, the piece length is P = max(min_len, mult * ceil(m)); a node with more
 * than P edges becomes ceil(deg / P) near-equal pieces, every other node one item, in
 * node order.  work holds 5 * max_items int32, max_items >= n + 2 * indptr[n] / min_len
 * + 1: the items (4 int32 each) and after them the zeroed counters; *count receives the
 * item count, or 0 when no node is longer than P (then the kernels walk the nodes as
 * before).  min_len <= 0: *count = 0.  One block; once per batch (the relation build). */
int hsg_rel_work(int n, const int32_t *indptr, int min_len, int mult, int32_t *work, int max_items,
                 int32_t *count, void *stream);
size_t hsg_rel_build_workspace_bytes(int n_nodes, int n_edges);
int hsg_rel_build(float src_unit, float dst_unit, int n_nodes, int n_edges, const int64_t *src,
                  const int64_t *dst, const float *unit, const int64_t *tffrac, const float *edtype,
                  int32_t *counts, int32_t *indptr, int32_t *esrc, uint8_t *tf, int64_t *eid,
                  int32_t *phantom, int32_t *cindptr, int32_t *cdst, int32_t *cperm,
                  int64_t *src_nodes, int64_t *dst_nodes, void *workspace, size_t workspace_bytes,
                  void *stream);

/* ---- sentence CNN encoder (module/Encoder.py:56-76) --------------------------------
 * Six Conv2d(1, 50, (h, D)), h = 2..7, + ReLU + max-pool over time, restated as one
 * GEMM Y = X Wall^T (hsg_gemm_f32; Wall [27*50][D], row (tap(h,i))*50 + c =
 * W_h[c][0][i][:], taps ordered h = 2..7, i = 0..h-1) plus a shifted sum.  X holds
 * only the rows a window can see: for sentence s, rows rowoff[s] .. rowoff[s]+len_s-1
 * are embed[ids[s][t]] + pos[t+1] and row rowoff[s]+len_s is the pad row embed[0] +
 * pos[0] (rowoff [n+1], rowoff[s+1]-rowoff[s] = len_s+1; padding must be trailing).
 *   hsg_cnn_gather:   builds X [rows][D].
 *   hsg_cnn_pool:     feat[s][(h-2)*50+c] = relu(max_t (b_h[c] + sum_i Y[row(s,t+i)][tap(h,i)*50+c]))
 *                     and arg = the first t of the max (CPU max_pool1d order); bias = 6
 *                     device pointers (host array).
 *   hsg_cnn_pool_bwd: adds dfeat (ReLU-masked) into the h rows of each max window of a
 *                     zero-filled dY [rows][lddy]; then dWall = dY^T X (hsg_gemm_f32).
 * hsg_cnn_taps() = 27*50 (columns of Y).  ldy, lddy >= 1350. */
int hsg_cnn_taps(void);
int hsg_cnn_gather(int n, int L, int D, const int64_t *ids, const float *embed, const float *pos,
                   const int32_t *rowoff, long rows, float *X, void *stream);
int hsg_cnn_pool(int n, int L, const int32_t *rowoff, const float *Y, int ldy, const float *const *bias,
                 float *feat, int32_t *arg, void *stream);
int hsg_cnn_pool_bwd(int n, const int32_t *rowoff, const float *feat, const int32_t *arg, const float *dfeat,
                     float *dY, int lddy, void *stream);

/* Library build identification (ABI version, gfx target). */
const char *hsg_version(void);

#ifdef __cplusplus
}
#endif
#endif /* HSG_H_ */
