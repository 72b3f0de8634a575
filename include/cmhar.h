/*
 * cmhar — C ABI of the MI355X (gfx950) HIP library behind the cross-modal IMU+video pretraining step.
 *
 * The reference (YOUNESELBOUKNIFY/CrossModal-IMU-Video-OOD-HAR) is pure Python: its hot path is the
 * `CrossModalModel` / `SigmoidContrastiveLoss` forward+backward driven by `CrossModalTrainer.train_epoch`
 * (src/train/trainer.py:130-144), executing through torch / transformers kernels.  There is no reference FFI;
 * each entry point below replaces one op family of that path, cited as "replaces: file:line".  The Python
 * host side (cmhar/_lib.py) binds these with ctypes; see INTEGRATION.md for the binding a maintainer would add.
 *
 * Conventions: all pointers are device pointers (HBM) unless stated; `stream` is a hipStream_t (the caller's
 * current stream); functions never allocate or synchronise — workspaces are passed in; return 0 on success,
 * a negative value for an unsupported argument combination, or a positive hipError_t from the launch.
 * dtype codes: 0 = fp32, 1 = bf16, 2 = fp16 (inference path only).  Matrices are row-major with explicit leading dimensions (elements).
 */
#ifndef CMHAR_H
#define CMHAR_H
#include <hip/hip_runtime_api.h>   /* hipStream_t only: the header is plain C */

#ifdef __cplusplus
extern "C" {
#endif

/* Fused GEMM epilogue (see csrc/common.h for the element formula). */
typedef struct CmharEpilogue {
  const float* bias;      /* [N] fp32 or NULL */
  const void* residual;   /* [M,N] output dtype, added last, or NULL */
  long ldr;
  const void* aux_in;     /* [M,N] pre-activation for act = 3 (dGELU) / 4 (dReLU); multiplier for act = 6 */
  long lda;
  void* aux_out;          /* [M,N] written by act = 1 (pre-activation) / act = 5 (GELU derivative) */
  long ldo;
  const float* rowadd;    /* [rowadd_mod, rowadd_ld] fp32 table added at row m % rowadd_mod */
  int rowadd_mod;
  int rowadd_ld;
  int act;                /* 0 none, 1 gelu(erf), 2 relu, 3 x*gelu'(aux_in), 4 x*(aux_in>0),
                             5 gelu(erf) with aux_out = gelu'(x) (the backward then needs only act 6),
                             6 x*aux_in */
  float alpha;            /* out = alpha*acc ... */
  float beta;             /* ... + beta*out_old (fp32 outputs; 0 = overwrite) */
  float pdrop;            /* element dropout after the activation (mask = hash(seed, m, n) >= pdrop), 0 = off */
  int pad_;
  unsigned long long seed;
  float* rowsum;          /* layout 2 (weight gradient) only: rowsum[m] = Σ_k A(m,k) + rowsum_beta·rowsum[m] —
                             the bias gradient Σ_tokens dY, taken from the same MFMA operand tiles; or NULL */
  float rowsum_beta;
  int colscale_lo;        /* columns [colscale_lo, colscale_hi) (multiples of 8) of alpha·acc + bias + rowadd are */
  int colscale_hi;        /* multiplied by colscale before the activation (the pre-scaled attention keys of the  */
  float colscale;         /* QKV projection); lo == hi: none */
} CmharEpilogue;

int cmhar_version(void);

/* bf16 MFMA GEMM (replaces: the nn.Linear forward/backward of the VideoMAE blocks, third-party
 * transformers modeling_videomae.py:209-324, the tubelet Conv3d :159-168 as an im2col GEMM, and
 * VideoEncoder.projection models.py:178,202).
 * layout 0: C = A[M,K] · B[N,K]ᵀ   1: C = A[M,K] · B[K,N]   2: C = A[K,M]ᵀ · B[K,N].
 * splits > 1: split-K with ws = splits*M*N (+ splits*M when epi->rowsum) fp32 floats.
 * epi->rowsum is supported on the 256-tile path (M, N % 256 == 0, K % 64 == 0) of layout 2; else returns -3. */
int cmhar_gemm_bf16(int layout, int out_dtype, int M, int N, int K, const void* A, long lda, const void* B, long ldb,
                    void* C, long ldc, const CmharEpilogue* epi, int splits, void* ws, hipStream_t stream);
/* Workspace (fp32 floats) a splits == 1 call may use: when the 256-tile count leaves the chip's last round less than
 * half full, the full rounds run whole-K and the remaining tile rows are split along K (partials in ws, reduced
 * with the epilogue).  0 = no workspace needed; a call with ws == NULL always runs whole-K. */
long cmhar_gemm_bf16_ws(int M, int N, int K);
/* The kernel plan cmhar_gemm_bf16 would run for these arguments (has_ws: ws != NULL; rowsum: epi->rowsum set):
 * 0 = 128² tile, 1 = 256² tile, 2 = 256² + tail split + reduce, 3 = 256² split-K + reduce, 4 = 8-phase 256²
 * (forward / weight-gradient layouts), 5 = 128² split-K + reduce, 6 = 8-phase 256² split-K + reduce (weight
 * gradients); -1 = bad layout.  Used for trace labels (bench.py kernel breakdown). */
int cmhar_gemm_bf16_plan(int layout, int M, int N, int K, int splits, int has_ws, int rowsum);
/* As cmhar_gemm_bf16_plan for a 16-bit output whose epilogue the persistent forward kernel takes (reads == 0: alpha
 * 1, no dropout / rowadd / beta; plain, the GELU pair, x aux_in or + residual) or not (reads != 0); 7 = the persistent
 * 8-phase forward kernel (whole-K forward-layout launches of at least three chip rounds of 256² tiles, an even K-tile
 * count, N <= 4096; at run time also 16-B aligned C / epilogue operands with leading dimensions % 8 == 0).
 * cmhar_gemm_bf16_plan answers for reads == 0.  A plan-7 launch with at least four K-tiles claims its tiles from a
 * 64-B counter block the library allocates (hipMalloc) on the first such launch per (device, stream) and keeps for
 * the process; each launch leaves it zeroed (CMHAR_PERSIST_DYNAMIC=0: the fixed tile walk, no allocation). */
int cmhar_gemm_bf16_plan2(int layout, int M, int N, int K, int splits, int has_ws, int rowsum, int reads);
/* cmhar_gemm_bf16 restricted to a phase mask: bit 0 = the GEMM kernel, bit 1 = the split-K / tail reduce (3 = the
 * whole call).  Calling phases 1 then 2 on one stream equals one cmhar_gemm_bf16 call; bench.py uses the split to
 * time the GEMM kernel alone with HIP events.  Returns -1 for phases outside 1..3. */
int cmhar_gemm_bf16_phased(int layout, int out_dtype, int M, int N, int K, const void* A, long lda, const void* B,
                           long ldb, void* C, long ldc, const CmharEpilogue* epi, int splits, void* ws,
                           hipStream_t stream, int phases);
/* fp16 MFMA GEMM, forward layout 0 only (C = A[M,K]·B[N,K]ᵀ, fp16 operands, out_dtype 2 = fp16 or 0 = fp32): the
 * fp16 inference path of BASELINE config 5 (replaces: the same VideoMAE nn.Linear / tubelet Conv3d forwards under
 * the reference's Evaluator.predict, src/eval/evaluator.py:28-53, run in half precision).  Arguments, workspace and
 * return codes as cmhar_gemm_bf16 (rowsum unsupported: -3; other layouts / dtypes: -1). */
int cmhar_gemm_f16(int layout, int out_dtype, int M, int N, int K, const void* A, long lda, const void* B, long ldb,
                   void* C, long ldc, const CmharEpilogue* epi, int splits, void* ws, hipStream_t stream);

/* Exact-fp32 (or mixed) strided batched GEMM: C[z][m,n] = epi(Σ_k A[z][m*sam+k*sak] B[z][k*sbk+n*sbn])
 * (replaces: the fp32 nn.Linear / IMU encoder / ProjectionHead matmuls, models.py:16-132, 221-234). */
int cmhar_gemm_generic(int in_dtype, int out_dtype, int M, int N, int K, int batch, const void* A, long sam,
                       long sak, long sAb, const void* B, long sbk, long sbn, long sBb, void* C, long ldc, long sCb,
                       const CmharEpilogue* epi, hipStream_t stream);
/* Split-K form of the above (batch 1) for skinny GEMMs with a long K (the video projection and projection heads at
 * M = batch rows): ws = splits*M*N fp32 partials, combined in a fixed order with the epilogue. */
int cmhar_gemm_generic_splitk(int in_dtype, int out_dtype, int M, int N, int K, int splits, const void* A, long sam,
                              long sak, const void* B, long sbk, long sbn, void* C, long ldc,
                              const CmharEpilogue* epi, float* ws, hipStream_t stream);

/* Attention softmax(scale·QKᵀ)V per (batch, head); Q/K/V/O rows [B*L, ld] with head h at cols h*D.
 * bf16: D = 64 flash kernels (no dropout).  fp16 (forward only; backward returns -1): the D = 64 flash kernel on
 * the fp16 MFMA, else the exact-f32-math kernel on fp16 storage.  fp32: D in {8,16,32,64}, attention-prob dropout pdrop.
 * lse: fp32 [B*H*Lq] (replaces: VideoMAESelfAttention modeling_videomae.py:209-258 and
 * nn.MultiheadAttention inside nn.TransformerEncoderLayer, models.py:85-95). */
int cmhar_attention_fwd(int dtype, int B, int H, int Lq, int Lk, int D, const void* Q, long ldq, const void* K,
                        long ldk, const void* V, long ldv, void* O, long ldo, float* lse, float scale, float pdrop,
                        unsigned long long seed, hipStream_t stream);
/* The bf16 / fp16 D = 64 flash forward's bulk launch: 1 = optimistic running max (frozen after a row's first 32
 * keys, no rescale) + an exact rerun of the workgroups whose rows left its range (the default; env
 * CMHAR_ATTN_FWD_OPT), 0 = one exact lazy-rescale launch.  mode < 0 only queries.  Returns the previous mode. */
int cmhar_attention_fwd_opt(int mode);
int cmhar_attention_bwd(int dtype, int B, int H, int Lq, int Lk, int D, const void* Q, long ldq, const void* K,
                        long ldk, const void* V, long ldv, const void* O, long ldo, const void* dO, long lddo,
                        const float* lse, float* delta, void* dQ, long lddq, void* dK, long lddk, void* dV, long lddv,
                        float scale, float pdrop, unsigned long long seed, hipStream_t stream);
/* bf16, D = 64 flash backward for PRE-SCALED keys (the VideoMAE training path): K holds bf16(scale·log2(e)·K),
 * written by the QKV GEMM's epilogue (CmharEpilogue.colscale over the key columns), and the forward was run with
 * scale = 1/log2(e) — so the recomputed scores are already in the exp2 domain and the per-score multiply is gone.
 * `scale` is the true softmax scale; dQ, dV and dK are the gradients of Q, V and the UNSCALED key (the QKV backward
 * is unchanged).  (replaces: the same VideoMAESelfAttention backward as cmhar_attention_bwd) */
int cmhar_attention_bwd_prescaled(int B, int H, int Lq, int Lk, const void* Q, long ldq, const void* K, long ldk,
                                  const void* V, long ldv, const void* O, long ldo, const void* dO, long lddo,
                                  const float* lse, float* delta, void* dQ, long lddq, void* dK, long lddk, void* dV,
                                  long lddv, float scale, hipStream_t stream);

/* y = LayerNorm(a + dropout(b)) (b nullable); h_out (nullable) receives a + dropout(b)
 * (replaces: VideoMAE layernorm_before/after modeling_videomae.py:337-350, IMU post-LN norm1/norm2 and
 * final norm models.py:85-95,127). */
int cmhar_layernorm_fwd(int dtype, int M, int N, const void* a, long lda, const void* b, long ldb, float pdrop,
                        unsigned long long seed, void* h_out, long ldh, void* y, long ldy, const float* gamma,
                        const float* beta, float* mean, float* rstd, float eps, hipStream_t stream);
long cmhar_layernorm_bwd_ws(int M, int N);
int cmhar_layernorm_bwd(int dtype, int M, int N, const void* dy, long lddy, const void* h, long ldh,
                        const float* gamma, const float* mean, const float* rstd, const void* dres, long ldres,
                        void* dh, long lddh, void* db_out, long lddb, float pdrop, unsigned long long seed,
                        float* dgamma, float* dbeta, float beta_acc, float* ws, hipStream_t stream);

/* out[n] = alpha Σ_m X[m,n] + beta out[n]  (bias gradients).  ws: cmhar_colsum_ws(M,N) floats. */
long cmhar_colsum_ws(int M, int N);
int cmhar_colsum(int dtype, int M, int N, const void* X, long ldx, float* out, float alpha, float beta, float* ws,
                 long ws_floats, hipStream_t stream);

/* BatchNorm1d (+ReLU) over [B,C] fp32 (replaces: ProjectionHead net.1/net.2 models.py:226-230,
 * IMUClassifier classifier models.py:317-320). */
int cmhar_batchnorm_fwd(int B, int C, const float* x, float* y, const float* w, const float* bias, float* rmean,
                        float* rvar, float* smean, float* srstd, int training, float momentum, float eps, int relu,
                        long long* num_batches_tracked, hipStream_t stream);
int cmhar_batchnorm_bwd(int B, int C, const float* x, const float* y, const float* dy, const float* w,
                        const float* smean, const float* srstd, float* dx, float* dw, float* db, int training,
                        int relu, float beta_acc, hipStream_t stream);

/* F.normalize(dim=1) (replaces: models.py:288-289). */
int cmhar_l2normalize_fwd(int M, int N, const float* x, float* y, float* norm, float eps, hipStream_t stream);
int cmhar_l2normalize_bwd(int M, int N, const float* y, const float* dy, const float* norm, float* dx, float eps,
                          hipStream_t stream);

/* SigmoidContrastiveLoss forward + gradients (replaces: src/models/losses.py:25-54). t, bias: device scalars.
 * ws: cmhar_siglip_ws(Ba,Bb) floats. */
long cmhar_siglip_ws(int Ba, int Bb);
int cmhar_siglip_loss(int Ba, int Bb, int D, const float* a, const float* b, const float* t, const float* bias,
                      float* loss, float* da, int a_off, int a_cnt, float* db, int b_off, int b_cnt, float* gt,
                      float* gbias, float* ws, hipStream_t stream);

/* VideoMAE tubelet patches (replaces: the Conv3d input side, modeling_videomae.py:159-168). */
int cmhar_tubelet_im2col(int out_dtype, int B, int T, int C, int H, int W, int tub, int P, const float* video,
                         void* out, hipStream_t stream);

/* IMU PatchTST embedding + CLS + positional truncation (replaces: models.py:30-50, 108-123).
 * w, bias, dw, db: HOST arrays of C device pointers. */
int cmhar_imu_embed_fwd(int B, int C, int L, int N, int P, int S, int D, int T, const float* x,
                        const float* const* w, const float* const* bias, const float* cls, const float* pos,
                        float* out, hipStream_t stream);
int cmhar_imu_embed_bwd(int B, int C, int L, int N, int P, int S, int D, int T, int Tpos, const float* x,
                        const float* dout, float* dcls, float* dpos, float* const* dw, float* const* db,
                        hipStream_t stream);

/* One post-LN nn.TransformerEncoderLayer of the IMU encoder (models.py:85-95 with d_model 128, 8 heads, FF 512):
 * parameters (fp32, torch layouts: in_proj [384,128], out_proj [128,128], linear1 [512,128], linear2 [128,512]) and
 * the activations the backward reads, written as [B*T, width] rows: qkv [.,384], o [.,128], lse [B*8*T], s1 = h +
 * drop(attn), mu1 / rs1 [B*T], h1 = LN1(s1), fd = drop(relu(linear1(h1))) [.,512], s2 = h1 + drop(linear2(fd)),
 * mu2 / rs2, h2 = LN2(s2). */
#define CMHAR_IMU_MAX_LAYERS 8
typedef struct CmharIMULayer {
  const float *w_qkv, *b_qkv, *w_out, *b_out, *ln1_g, *ln1_b, *w_ff1, *b_ff1, *w_ff2, *b_ff2, *ln2_g, *ln2_b;
  float eps1, eps2;
  float *qkv, *o, *lse, *s1, *mu1, *rs1, *h1, *fd, *s2, *mu2, *rs2, *h2;
} CmharIMULayer;
/* The IMU encoder's transformer stack + final LayerNorm in ONE launch (replaces: IMUEncoder.forward's
 * self.transformer(x) and self.norm(x), models.py:125-130): one workgroup per window keeps its T <= 32 token rows in
 * LDS through all `nlayers` (<= CMHAR_IMU_MAX_LAYERS) layers.  x: [B*T, 128] embedded tokens; layers: HOST array;
 * enc = norm(h2 of the last layer) with its mean / rstd.  Dropout (pdrop, layer i's streams from seed + 7919(i+1))
 * as the separate kernels; every output is bit-identical to the per-op launches (cmhar_gemm_generic,
 * cmhar_attention_fwd, cmhar_layernorm_fwd).  Returns -1 for other geometries (D != 128, H != 8, FF != 512, T > 32). */
int cmhar_imu_encoder_fwd(int B, int T, int D, int H, int FF, int nlayers, const float* x, const CmharIMULayer* layers,
                          const float* norm_g, const float* norm_b, float norm_eps, float* enc, float* norm_mu,
                          float* norm_rs, float scale, float pdrop, unsigned long long seed, hipStream_t stream);
/* Per-layer outputs of the fused backward: token-gradient scratch [B*T, width] (dqkv 384, da 128, dpre 512, df2 128,
 * gln1 / gln2 = the incoming gradients of norm1 / norm2, 128) and the parameter gradients (parameter shapes). */
typedef struct CmharIMULayerGrad {
  float *dqkv, *da, *dpre, *df2, *gln1, *gln2;
  float *dw_qkv, *db_qkv, *dw_out, *db_out, *dln1_g, *dln1_b, *dw_ff1, *db_ff1, *dw_ff2, *db_ff2, *dln2_g, *dln2_b;
} CmharIMULayerGrad;
/* Backward of cmhar_imu_encoder_fwd (replaces: autograd through models.py:125-130) from the tensors it saved
 * (layers: the same array; x: its input) and d_enc = dL/d(encoded tokens) [B*T, 128]: dx [B*T, 128] for the
 * embedding backward, every layer's parameter gradients (grads, nlayers entries) and the final norm's (dnorm_g,
 * dnorm_b).  Two launches: one workgroup per window runs the token-gradient chain through all layers (dgrads and
 * attention backward bit-identical to the per-op launches); one grouped launch forms every weight gradient (the
 * same token-ordered chain as the weight-gradient GEMM) and the bias / affine column sums (sequential over tokens;
 * the per-op path sums in two levels, so these differ from it by rounding only). */
int cmhar_imu_encoder_bwd(int B, int T, int D, int H, int FF, int nlayers, const float* x, const CmharIMULayer* layers,
                          const CmharIMULayerGrad* grads, const float* norm_g, const float* norm_mu,
                          const float* norm_rs, const float* d_enc, float* dnorm_g, float* dnorm_b, float* dx,
                          float scale, float pdrop, unsigned long long seed, hipStream_t stream);

/* dst[r, c] = alpha * src[r, c] * dropmask(seed, pdrop, r, c) + beta * dst[r, c], with dtype conversion
 * (token-0 gather, casts, gradient adds, nn.Dropout forward/backward, models.py:85-95, 311-322). */
int cmhar_copy2d(int in_dtype, int out_dtype, int rows, int cols, const void* src, long lds, void* dst, long ldd,
                 float alpha, float beta, float pdrop, unsigned long long seed, hipStream_t stream);

/* Energy-score OOD head over classifier logits [N, C] (row stride ld): pred[i] = first argmax, maxlogit[i],
 * energy[i] = -T * logsumexp(logits[i] / T)  (no reference counterpart — SURVEY §8(f) rank 1; the logits are those
 * of Evaluator.predict, src/eval/evaluator.py:28-53).  Outputs are nullable. */
int cmhar_logits_energy(int dtype, int N, int C, const void* logits, long ld, float temperature, int* pred,
                        float* energy, float* maxlogit, hipStream_t stream);

/* Row-softmax cross-entropy family over the strided logit view z[r][c] = logits[r*s_row + c*s_col], r < N, c < C
 * (replaces: nn.CrossEntropyLoss, ClassificationTrainer trainer.py:249,300; FocalLoss losses.py:90-116;
 * LabelSmoothingCrossEntropy losses.py:119-150; both F.cross_entropy of InfoNCELoss losses.py:76-85).
 * labels: device int64 [N] or NULL (= row index); rows whose label == ignore_index are skipped.  gamma/alpha: focal
 * weighting (gamma = 0, alpha = 1: plain CE; label_smoothing and gamma are exclusive).  reduction 0 none / 1 mean /
 * 2 sum.  Outputs (all nullable): loss scalar, row_loss [N], pred (first argmax) [N], correct = #(pred == label),
 * status = 1 when a label is out of range (the host raises).  dlogits (nullable, strides d_row/d_col):
 * dlogits = grad_beta*dlogits + grad_scale*g*dloss/dz, g = g_up[r] ('none', required) or (*g_up or 1) x (1/count
 * for 'mean').  ws: cmhar_cross_entropy_ws(N) floats. */
long cmhar_cross_entropy_ws(int N);
int cmhar_cross_entropy(int N, int C, const float* logits, long s_row, long s_col, const long* labels,
                        long ignore_index, float label_smoothing, float gamma, float alpha, int reduction, float* loss,
                        float* row_loss, long* pred, int* correct, int* status, float* dlogits, long d_row, long d_col,
                        float grad_scale, float grad_beta, const float* g_up, float* ws, hipStream_t stream);

/* Video clip ingestion (replaces: CrossModalDataset.load_video_clip + its transform, src/data/datasets.py:49-58,
 * 155-235): decoded RGB uint8 frames [*][H0][W0][3] (frame f at frames + f*frame_stride bytes), frame_idx: device
 * int32 [B*T] source frame per output frame → out fp32 (B,T,3,H,W) (channel_first = 0) or (B,3,T,H,W), each
 * frame resized with Pillow's BILINEAR resample bit-exactly (22-bit fixed point, uint8 between the passes), then
 * /255 and (x - mean)/std.  mean3/std3: HOST arrays of 3 floats.  ws: cmhar_video_ingest_ws(B*T, H0, W0, H, W) bytes. */
int cmhar_resize_ksize(int in_size, int out_size);
long cmhar_video_ingest_ws(int nframes, int H0, int W0, int H, int W);
int cmhar_video_ingest(int B, int T, const unsigned char* frames, long frame_stride, int H0, int W0,
                       const int* frame_idx, int H, int W, const float* mean3, const float* std3, int channel_first,
                       float* out, void* ws, long ws_bytes, hipStream_t stream);

/* IMU preprocessing (replaces: MMEAPreprocessor.load_imu_data unit conversion, preprocess_imu, create_imu_windows,
 * src/data/preprocessing.py:176-183, 204-243).  raw: [total][C] fp32, recording r = rows offsets[r]..offsets[r+1]
 * (device int64 [nrec+1]); div_r: device [C] unit divisors (raw / R) or NULL; median_k odd (1 = off; zero-padded
 * edges like scipy.signal.medfilt); normalize: per-recording per-channel z-score, population std + 1e-8.
 * Windows w < nwin: recording win_rec[w] (device int32), first sample win_start[w] (device int64), win samples,
 * zero past the recording's end → out [nwin][C][win] fp32.  ws: cmhar_imu_preprocess_ws(total, nrec, C) floats. */
long cmhar_imu_preprocess_ws(long total, int nrec, int C);
int cmhar_imu_preprocess(int nrec, int C, const float* raw, const long* offsets, long total, const float* div_r,
                         int median_k, int normalize, long nwin, const int* win_rec, const long* win_start, int win,
                         float* out, float* ws, hipStream_t stream);

/* Multi-tensor optimizer (replaces: torch.nn.utils.clip_grad_norm_ and torch.optim.AdamW.step,
 * trainer.py:74-78,140-141).  tens/chunks: DEVICE arrays of
 *   struct { float* p; const float* g; float* m; float* v; bf16* p_bf16; float* p_copy; long n; float wd;
 *            float lr_scale; }      (p_bf16 / p_copy: optional compute shadows refreshed in the same pass)
 *   struct { int tensor; int pad; long start; long len; }
 * grad_norm: out[0] = total L2 norm, out[1] = min(1, max_norm/(norm+1e-6)); apply_clip scales grads in place.
 * adamw: step scalars precomputed by the host in double (torch semantics); gscale (nullable) = out of grad_norm. */
int cmhar_mt_grad_norm(const void* tens, const void* chunks, int nchunks, float* part, float* out, float max_norm,
                       int apply_clip, hipStream_t stream);
int cmhar_mt_adamw(const void* tens, const void* chunks, int nchunks, float lr, float one_minus_beta1, float beta2,
                   float one_minus_beta2, float eps, float step_size, float bias_correction2_sqrt,
                   const float* gscale, hipStream_t stream);
/* cmhar_mt_adamw with the gradient clipping folded in (FusedAdamW(max_grad_norm=...)): the gradient is scaled by the
   device-side clip coefficient gscale[1] written by cmhar_mt_grad_norm(apply_clip = 0), replacing the separate
   in-place scale pass of trainer.py:140 clip_grad_norm_; write_grad != 0 also stores the clipped gradient back into
   .grad in the same pass (torch's post-clip .grad).  Same update, bit for bit, as clip-then-step. */
int cmhar_mt_adamw_clip(const void* tens, const void* chunks, int nchunks, float lr, float one_minus_beta1,
                        float beta2, float one_minus_beta2, float eps, float step_size, float bias_correction2_sqrt,
                        const float* gscale, int write_grad, hipStream_t stream);
/* refresh the compute shadows (p_bf16 / p_copy) from p, e.g. after a foreign optimizer updated p. */
int cmhar_mt_cast_bf16(const void* tens, const void* chunks, int nchunks, hipStream_t stream);
/* Transposed bf16 copies of weight shadows (the input-gradient GEMMs' forward-layout operand Wᵀ): descs = ndesc
 * records {const bf16* src; bf16* dst; int rows; int cols; int tile0; int pad;} (32 B; src [rows, cols] → dst
 * [cols, rows], rows and cols multiples of 8, tile0 = first 64×64 tile of the record, ascending), ntiles = total. */
int cmhar_mt_transpose_bf16(const void* descs, int ndesc, int ntiles, hipStream_t stream);

/* ---- R3D-18 video backbone (north_star extension; no reference code — the reference's CNN options are per-frame
 * 2-D torchvision models, models.py:160-216; replaces torchvision.models.video.r3d_18's Conv3d / BatchNorm3d /
 * AdaptiveAvgPool3d).  Activations are channels-last NDHWC.  dims: HOST int[15] =
 * {N, T, H, W, C, kt, kh, kw, st, sh, sw, pt, ph, pw, Kp}; col is [N·To·Ho·Wo, Kp] with k = ((it·kh+ih)·kw+iw)·C + c
 * (zero for k >= kt·kh·kw·C); the convolution itself is cmhar_gemm_bf16 / cmhar_gemm_generic over col. */
int cmhar_conv3d_im2col(int in_dtype, int out_dtype, const int* dims, const void* x, void* col, hipStream_t stream);
/* Implicit-GEMM convolution on MFMA (bf16, C % 64 == 0, Kp == kt·kh·kw·C; no column matrix in HBM):
 * z [M, Cout] = col(x) · Wᵀ (+ res [M, Cout], nullable) with W [Cout, Kp] in the im2col k order — also the input
 * gradient of a stride-1 conv (x = dz, W = the tap-flipped, in/out-transposed weight); dw [Cout, Kp] fp32 =
 * dzᵀ · col(x), split over M into ws (cmhar_conv3d_wgrad_ws floats; 0 = no workspace), reduced in a fixed order. */
int cmhar_conv3d_fwd(const int* dims, int Cout, const void* x, const void* w, const void* res, void* z,
                     float* tile_stats, hipStream_t stream);
/* The kernel cmhar_conv3d_fwd launches for a geometry (tests pin the production plans): 1 = nine-tap row slab
 * (Cout = 64), 2 / 3 = row slab with 128- / 256-row tiles, 4 / 5 = generic gather with 128x64 / 128x128 tiles;
 * -1 = not an implicit-GEMM geometry.  cmhar_conv3d_wgrad_plan likewise for cmhar_conv3d_wgrad: 1 = nine-tap row
 * slab, 2 / 3 = row slab with 128- / 64-wide Cout tiles, 4 = generic gather (split reduce when its ws > 0). */
int cmhar_conv3d_fwd_plan(const int* dims, int Cout);
int cmhar_conv3d_wgrad_plan(const int* dims, int Cout);
/* Split-K forward for the convs whose output tile grid leaves most of the chip idle (R3D-18 layer 4): ws fp32
 * floats = cmhar_conv3d_fwd_split_ws(dims, Cout) (0: not this plan — call cmhar_conv3d_fwd); z = conv(x) (+ res),
 * no BatchNorm tile statistics (the caller's BatchNorm takes its own statistics passes). */
long cmhar_conv3d_fwd_split_ws(const int* dims, int Cout);
int cmhar_conv3d_fwd_split(const int* dims, int Cout, const void* x, const void* w, const void* res, void* z, float* ws,
                           hipStream_t stream);
/* tile_stats (nullable): per row tile of z and channel, the mean and Σ(v − mean)² of the bf16 outputs and each
 * tile's row count, consumed by cmhar_bn_cl_fwd_tiles (training-mode BatchNorm3d of z without a statistics pass).
 * cmhar_conv3d_fwd_tiles gives the tile count ntile of the forward's plan (-1: not an implicit-GEMM conv) and
 * cmhar_conv3d_fwd_stats_floats the buffer size: [2][ntile][Cout] tile partials | [2][ngroup][Cout] group partials
 * | [ntile] tile row counts | [ngroup] group row counts, ngroup = ceil(ntile/16). */
int cmhar_conv3d_fwd_tiles(const int* dims, int Cout);
long cmhar_conv3d_fwd_stats_floats(const int* dims, int Cout);
int cmhar_bn_cl_fwd_tiles(long M, int C, int ntile, float* tile_stats, const void* x, const void* res, void* y,
                          const float* w, const float* b, float* rmean, float* rvar, float* smean, float* srstd,
                          float momentum, float eps, int relu, long long* num_batches_tracked, hipStream_t stream);
/* Implicit stem convolution for few input channels (C <= 4), kw <= 8 at w-stride 2, Cout = 64 — R3D-18's BasicStem
 * Conv3d(3, 64, (3,7,7), (1,2,2), (1,3,3)) and ResNet-18's 7x7/2 stem, replacing their im2col + GEMM (replaces: the
 * stem nn.Conv3d / nn.Conv2d of torchvision r3d_18 / resnet18, models.py:160-216).  Weights packed by
 * cmhar_conv_pack_stem as [Cout][kt][kh][32] bf16, element iw·4 + c (zero past kw / C); z = [M][64] bf16 with
 * tile statistics as cmhar_conv3d_fwd's (sized by cmhar_conv3d_stem_tiles / cmhar_conv3d_stem_stats_floats; -1:
 * geometry not supported); the weight gradient is written fp32 in the packed layout, with ws =
 * cmhar_conv3d_stem_wgrad_ws floats. */
int cmhar_conv3d_stem_tiles(const int* dims, int Cout);
long cmhar_conv3d_stem_stats_floats(const int* dims, int Cout);
int cmhar_conv_pack_stem(int Cout, int C, int kt, int kh, int kw, const float* w, void* out, hipStream_t stream);
int cmhar_conv3d_stem_fwd(const int* dims, int Cout, const void* x, const void* w4, void* z, float* tile_stats,
                          hipStream_t stream);
long cmhar_conv3d_stem_wgrad_ws(const int* dims, int Cout);
int cmhar_conv3d_stem_wgrad(const int* dims, int Cout, const void* x, const void* dz, float* dw4, float* ws,
                            hipStream_t stream);
long cmhar_conv3d_wgrad_ws(const int* dims, int Cout);
int cmhar_conv3d_wgrad(const int* dims, int Cout, const void* x, const void* dz, float* dw, float* ws,
                       hipStream_t stream);
/* dx (NDHWC, dtype) = Σ over taps of dcol (+ dx when accumulate): the input gradient of the convolution. */
int cmhar_conv3d_col2im(int dtype, const int* dims, const void* dcol, void* dx, int accumulate, hipStream_t stream);
/* BatchNorm3d / BatchNorm2d over the [M, C] channels-last view (C % 8 == 0, C ≤ 2048, M < 2^31), fused residual add
 * + activation: y = act(bn(x) + res), relu 0 = none, 1 = ReLU, 2 = ReLU6 (MobileNetV2).  ws: cmhar_bn_cl_ws(M, C) floats.  Training updates rmean/rvar/num_batches_tracked. */
long cmhar_bn_cl_ws(long M, int C);
int cmhar_bn_cl_fwd(int dtype, long M, int C, const void* x, const void* res, void* y, const float* w,
                    const float* b, float* rmean, float* rvar, float* smean, float* srstd, int training,
                    float momentum, float eps, int relu, long long* num_batches_tracked, float* ws,
                    hipStream_t stream);
/* g = dy·act'(y) ([y > 0] for relu 1, [0 < y < 6] for relu 2); dres = g (optional); dx = BN input gradient; dw = Σg·x̂, db = Σg (fp32, overwritten). */
int cmhar_bn_cl_bwd(int dtype, long M, int C, const void* x, const void* y, const void* dy, const float* w,
                    const float* smean, const float* srstd, void* dx, void* dres, float* dw, float* db, int training,
                    int relu, float* ws, hipStream_t stream);
/* The same for a unit whose forward added no residual (y = act(bn(x))): act'(y) is recomputed from x with b in the
 * forward's exact arithmetic and rounding (the same mask bit for bit), so y is not read; no dres. */
int cmhar_bn_cl_bwd_nores(int dtype, long M, int C, const void* x, const void* dy, const float* w, const float* b,
                          const float* smean, const float* srstd, void* dx, float* dw, float* db, int training,
                          int relu, float* ws, hipStream_t stream);
/* AdaptiveAvgPool3d(1): [N, S, C] → fp32 [N, C], and its backward (dx = dout / S broadcast). */
int cmhar_avgpool_cl(int dtype, int N, long S, int C, const void* x, float* out, hipStream_t stream);
int cmhar_avgpool_cl_bwd(int dtype, int N, long S, int C, const float* dout, void* dx, hipStream_t stream);
/* Weight packs for the conv kernels, from the fp32 master w [Cout, Cin, kt, kh, kw] in one pass (either output
 * nullable): out [Cout, Kp] (out_dtype) in the im2col k order ((it·kh + ih)·kw + iw)·Cin + ci, zero for k ≥ K;
 * out_flip [Cin, taps·Cout]: the tap-flipped, in/out-transposed weight (k = tap·Cout + co) the stride-1 input
 * gradient convolves dz with.  taps = kt·kh·kw ≤ 384. */
int cmhar_conv_pack_weight(int out_dtype, int Cout, int Cin, int kt, int kh, int kw, int Kp, const float* w,
                           void* out, void* out_flip, hipStream_t stream);
/* n such packs in one launch: dims host [n][6] = (Cout, Cin, kt, kh, kw, Kp), ptrs host [n][3] = (w, out, out_flip),
 * the same arguments and outputs as n cmhar_conv_pack_weight calls. */
int cmhar_conv_pack_weights(int out_dtype, int n, const int* dims, const void* const* ptrs, hipStream_t stream);
/* Weight gradient from a packed k order back to the parameter layout (replaces the strided-view copy autograd's
 * gradient accumulation made of the conv weight gradient, torchvision conv weights [Cout, Cin, kt, kh, kw]):
 * dst [Cout, Cin, R, kw] fp32 (R = kt·kh) from src [Cout, Kp] fp32 at co·Kp + r·rs + iw·cs + ci — im2col order
 * rs = kw·Cin, cs = Cin; implicit stem rs = 32, cs = 4.  -2: Cout·Cin·R·kw too large. */
int cmhar_conv_grad_unpack(int Cout, int Cin, int R, int kw, int Kp, int rs, int cs, const float* src, float* dst,
                           hipStream_t stream);

/* ---- per-frame 2-D CNN video backbones (replaces: torchvision resnet18 children[:-2] / mobilenet_v2 .features under
 * VideoEncoder, models.py:163-173,208-216).  Dense Conv2d = the conv3d entry points above with kt = 1; BatchNorm2d =
 * cmhar_bn_cl_* (relu 2 = ReLU6).  Activations NHWC [N, H, W, C], C % 8 == 0, window k·k ≤ 9, 2p ≤ k.
 * MaxPool2d(k, s, p): argmax = uint8 [N, Ho, Wo, C] tap index of the first maximum (torch's tie rule); the backward
 * gathers dy into dx (overwritten). */
int cmhar_maxpool2d_cl_fwd(int dtype, int N, int H, int W, int C, int k, int s, int p, const void* x, void* y,
                           unsigned char* argmax, hipStream_t stream);
int cmhar_maxpool2d_cl_bwd(int dtype, int N, int H, int W, int C, int k, int s, int p, const void* dy,
                           const unsigned char* argmax, void* dx, hipStream_t stream);
/* Depthwise Conv2d(C, C, k, s, p, groups = C, bias = False); w = the fp32 parameter [C, 1, k, k].  dgrad overwrites
 * dx; wgrad overwrites dw (fp32 [C, k, k]) through ws (cmhar_dwconv2d_cl_wgrad_ws floats), fixed-order sums. */
int cmhar_dwconv2d_cl_fwd(int dtype, int N, int H, int W, int C, int k, int s, int p, const void* x, const float* w,
                          void* z, hipStream_t stream);
int cmhar_dwconv2d_cl_dgrad(int dtype, int N, int H, int W, int C, int k, int s, int p, const void* dz,
                            const float* w, void* dx, hipStream_t stream);
long cmhar_dwconv2d_cl_wgrad_ws(int N, int H, int W, int C, int k, int s, int p);
int cmhar_dwconv2d_cl_wgrad(int dtype, int N, int H, int W, int C, int k, int s, int p, const void* x, const void* dz,
                            float* dw, float* ws, hipStream_t stream);

/* (B, T, C, H, W) fp32 clip batch → (B, T, H, W, C) in the compute dtype (the backbone's input layout). */
int cmhar_video_to_ndhwc(int out_dtype, int B, int T, int C, int H, int W, const float* video, void* out,
                         hipStream_t stream);

/* ---- measurement (the on-box MFMA peak).  Back-to-back bf16 MFMAs on random bf16 fragments, 8
 * independent chains per wave — shape 0: v_mfma_f32_32x32x16_bf16, 1: v_mfma_f32_16x16x32_bf16 (-1 otherwise):
 * `blocks` workgroups of 256 threads, `iters` iterations of 8 MFMAs per wave; ops = nops 16-B bf16 fragments
 * (random), out = blocks·256 floats.  _flops = the FLOPs one launch executes. */
long cmhar_mfma_peak_probe_flops(int shape, int blocks, int iters);
int cmhar_mfma_peak_probe(int shape, int blocks, int iters, const void* ops, int nops, float* out,
                          hipStream_t stream);

/* ---- plain library GEMMs on hipBLASLt (replaces: the VideoMAE attention output projection `nn.Linear`,
 * modeling_videomae.py VideoMAESelfOutput.dense, and its input gradient; reached from models.py:199).
 * out[M,N] = A[M,K]·B[N,K]ᵀ (+ bias[N] fp32) (+ residual[M,N]), fp32 accumulation, dtype CMHAR_BF16 or CMHAR_F16
 * (operands, residual and output); row-major operands
 * with leading dimensions lda / ldb / ldo / ldr (elements).  Plans (descriptor, layouts, heuristic algorithm) are
 * cached per shape and epilogue; a 128-MiB workspace per (device, stream), allocated on first use.  _ok: 1 when hipBLASLt has an algorithm for it. */
int cmhar_blaslt_linear(int dtype, int M, int N, int K, const void* A, long lda, const void* B, long ldb, void* out, long ldo,
                        const float* bias, const void* residual, long ldr, hipStream_t stream);
int cmhar_blaslt_linear_ok(int dtype, int M, int N, int K, long lda, long ldb, long ldo, int has_bias, int has_residual, long ldr);

#ifdef __cplusplus
}
#endif
#endif /* CMHAR_H */
