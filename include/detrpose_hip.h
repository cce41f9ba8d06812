/*
 * detrpose_hip.h — C ABI of libdetrpose_hip.so, the MI355X (gfx950) kernels of the
 * DETRPose inference forward.
 *
 * The reference has no native code and no FFI (SURVEY.md §1 key fact 1): its forward
 * is DETRPose.forward (src/models/detrpose/detrpose.py:76-81) built from torch leaf
 * ops. Each entry point below replaces one of those leaf ops / fused op groups; the
 * comment on each names the reference code it stands in for. The Python host in
 * detrpose_amd/ binds these with ctypes (detrpose_amd/_lib.py); INTEGRATION.md shows
 * the binding a maintainer adds to the reference.
 *
 * Conventions
 *  - Activations are channels-last (NHWC). Element (b, y, x, c) of a map lives at
 *    base + b*bstride + (y*w + x)*pstride + c  (elements, not bytes), so a kernel can
 *    read/write a channel slice of a wider concat buffer in place.
 *  - dtype: DP_F32 (parity mode) or DP_BF16 (bf16 storage, fp32 accumulation).
 *    Small decoder-head tensors (reference points, corners, logits) are always f32.
 *  - Every call enqueues asynchronously on `stream` (a hipStream_t) and never
 *    allocates device memory or synchronises. Buffers belong to the caller.
 *  - Return 0 on success; non-zero is a hipError_t or DP_EINVAL, with a message in
 *    dp_last_error(). Calls are stateless and re-entrant per stream.
 */
#ifndef DETRPOSE_HIP_H
#define DETRPOSE_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { DP_F32 = 0, DP_BF16 = 1 };
enum { DP_ACT_NONE = 0, DP_ACT_RELU = 1, DP_ACT_SILU = 2, DP_ACT_GELU = 3 };
enum { DP_EINVAL = 1000 };

/* Descriptor of one convolution / linear layer run as an implicit GEMM:
 * M = batch*out_h*out_w rows, N = cout, K = kh*kw*cin (k = (ky*kw + kx)*cin + c). */
typedef struct dp_conv_desc {
  const void* in;  int64_t in_bstride;  int32_t in_pstride;  int32_t in_h, in_w, cin;
  const void* weight;  int32_t kpad;      /* [cout][kpad] of dtype, zero padded in k */
  const float* bias;                      /* [cout] (folded BN shift) or NULL        */
  int32_t kh, kw, stride, pad_t, pad_l;
  void* out;       int64_t out_bstride; int32_t out_pstride; int32_t out_h, out_w, cout;
  const void* res; int64_t res_bstride; int32_t res_pstride;  /* added after act, or NULL */
  int32_t batch;
  int32_t act;     int32_t has_lab;  float lab_scale, lab_bias;  /* y = lab(act(x)) + res */
  int32_t dtype;
  /* up != NULL: also write a nearest x2 copy of the output to up (concat buffer slice) */
  void* up;        int64_t up_bstride;  int32_t up_pstride;
  /* out_f32 != 0: out (and res) are f32 whatever dtype is (1x1 / linear layers only) */
  int32_t out_f32;
  /* in_seg_ch != 0 (bf16 1x1 convs): the input's channels are cin / in_seg_ch segments of
   * in_seg_ch channels, segment s a map of its own at in + s * in_seg_stride elements (each
   * with in_pstride / in_bstride): the HG-block concat stored one contiguous map per layer */
  int32_t in_seg_ch;
  int64_t in_seg_stride;
} dp_conv_desc;

/* Row map: row r -> element offset  base + (r / group)*stride_g + (r % group)*stride_r. */
typedef struct dp_rowmap {
  int64_t base;  int32_t group;  int64_t stride_g;  int64_t stride_r;
} dp_rowmap;

const char* dp_last_error(void);
int dp_version(void);
/* Content hash of the sources this library was built from (detrpose_amd/build.py bakes it in;
 * the Python loader refuses a library whose hash differs from the shipped sources). */
const char* dp_source_hash(void);

/* The kernel instantiation dp_conv2d would launch for *d, written to buf (no launch, no
 * device access), in the demangled form rocprofv3 prints, e.g.
 * "conv_halo_kernel<8, 4, 3, 3, 1, 128, false, false, 2, false, 0>". For per-kernel roofline
 * accounting (bench.py). Returns 0, or DP_EINVAL for a descriptor dp_conv2d would refuse. */
int dp_conv2d_describe(const dp_conv_desc* d, char* buf, int32_t buflen);

/* nn.Conv2d (+ folded BatchNorm / FrozenBatchNorm2d) + act (+ LAB) (+ residual),
 * dense groups=1. Replaces ConvBNAct (hgnetv2.py:82-134), ConvNormLayer(_fuse)
 * (hybrid_encoder.py:56-128), VGGBlock deploy conv (139-189) and every nn.Linear of
 * the path (as a 1x1 conv over rows). MFMA implicit GEMM. */
int dp_conv2d(const dp_conv_desc* d, void* stream);

/* Depthwise conv (groups == channels) + folded BN + act: LightConvBNAct.conv2
 * (hgnetv2.py:137-166), HG_Stage downsample (349-358), SCDown.cv2
 * (hybrid_encoder.py:130-137). weight is f32 [kh][kw][C]. */
int dp_dwconv2d(const dp_conv_desc* d, void* stream);

/* StemBlock.stem1 (hgnetv2.py:171-177): 3x3 s2 p1 conv over the f32 NCHW image,
 * folded FrozenBN, ReLU (+ LAB); writes NHWC dtype. weight f32 [cout][3][3][3]. */
int dp_stem_conv(const float* image, int32_t batch, int32_t h, int32_t w,
                 const float* weight, const float* bias, int32_t cout,
                 int32_t has_lab, float lab_scale, float lab_bias,
                 void* out, int64_t out_bstride, int32_t out_pstride, int32_t dtype, void* stream);

/* Packed StemBlock weights for dp_stem_fused: stem1 f32 [32][27] (OIHW flattening), the
 * other convs bf16 [cout][k*] (k = tap * cin + ci, rows padded to k* elements) as dp_conv2d
 * takes them; stem3's cin is the cat order [pool, stem2b]. f32 biases (folded BN). LAB
 * (scale, bias) per conv in the order stem1, 2a, 2b, 3, 4 when has_lab. */
typedef struct dp_stem_weights {
  const float* w1;
  const float* b1;
  const void* w2a;
  const float* b2a;
  const void* w2b;
  const float* b2b;
  const void* w3;
  const float* b3;
  const void* w4;
  const float* b4;
  int32_t k2a, k2b, k3, k4;
  int32_t mid, cout;
  int32_t has_lab;
  float lab[5][2];
} dp_stem_weights;

/* The whole StemBlock.forward (hgnetv2.py:204-220: stem1, stem2a, stem2b, max-pool, cat,
 * stem3, stem4) in one bf16 launch: f32 NCHW image in, stem4's NHWC bf16 map out (into the
 * first HG stage's concat slot). Stem channels [3, 32, 48|64] (B4 / B5). Same rounding points
 * as the five-launch path (bit-identical output). */
int dp_stem_fused(const float* image, int32_t batch, int32_t h, int32_t w, const dp_stem_weights* weights,
                  void* out, int64_t out_bstride, int32_t out_pstride, void* stream);

/* F.pad(x,(0,1,0,1)) + MaxPool2d(2, 1, ceil_mode=True) of StemBlock (hgnetv2.py:215,217). */
int dp_maxpool2x2_pad_rb(const void* in, int64_t in_bstride, int32_t in_pstride,
                         int32_t batch, int32_t h, int32_t w, int32_t c,
                         void* out, int64_t out_bstride, int32_t out_pstride, int32_t dtype, void* stream);

/* dp_conv2d of StemBlock.stem2a (2x2 s1 over F.pad(x,(0,1,0,1)): pad 0, zero read past the
 * right/bottom edge) that also writes MaxPool2d(2, 1, ceil_mode=True) of the same padded
 * input to pool_out (hgnetv2.py:213-220): replaces the stem2a conv + dp_maxpool2x2_pad_rb pair
 * with one pass over stem1's output. bf16, cin % 8 == 0, cin <= 64, cout <= 32. */
int dp_conv2d_pool(const dp_conv_desc* d, void* pool_out, int64_t pool_bstride, int32_t pool_pstride,
                   void* stream);

/* out[r] = a[r] + b[r] over `rows` rows of `c` elements (row maps as above); b == NULL copies a. */
int dp_add_rows(void* out, dp_rowmap om, const void* a, dp_rowmap am, const void* b, dp_rowmap bm,
                int32_t rows, int32_t c, int32_t dtype, void* stream);

/* out = LayerNorm(x + res) (+ post on rows selected by post map).  nn.LayerNorm with
 * the residual adds of TransformerEncoderLayer (hybrid_encoder.py:281-296) and the
 * decoder layer (transformer.py:405-442).  row_mask/mask_period/masked_row: rows whose
 * mask[r % period] != 0 output masked_row (f32 [c]) instead: Transformer two-stage
 * masked_fill + enc_output + LN of a zero row (transformer.py:1232-1236). */
int dp_layernorm(void* out, dp_rowmap om, const void* x, dp_rowmap xm, const void* res, dp_rowmap rm,
                 const float* gamma, const float* beta, float eps, int32_t rows, int32_t c,
                 const void* post, dp_rowmap pm, int32_t post_group, int32_t post_skip,
                 const uint8_t* row_mask, int32_t mask_period, const float* masked_row,
                 int32_t dtype, void* stream);

/* Gate.forward (transformer.py:222-235) after its Linear: gates/xcat are [rows][2c]
 * ([x1 | x2]); out = LN(sigmoid(g1)*x1 + sigmoid(g2)*x2). */
int dp_gate_layernorm(void* out, int32_t out_ld, const void* gates, const void* xcat,
                      const float* gamma, const float* beta, float eps, int32_t rows, int32_t c,
                      int32_t dtype, void* stream);

/* Scaled dot-product attention core of nn.MultiheadAttention (batch_first, no mask,
 * eval): softmax(QK^T/sqrt(dh))V per head.  Sequence s = (o, i), o < n_outer,
 * i < n_inner; token t of it is row o*so + i*si + t*st of q/k/v (leading dims ld_q,
 * ld_kv) and of out (ld_o).  Within-/across-instance attention (transformer.py:
 * 403-419) and AIFI (hybrid_encoder.py:276-279). */
int dp_attention(const void* q, int32_t ld_q, const void* k, const void* v, int32_t ld_kv,
                 void* out, int32_t ld_o, int32_t n_outer, int32_t n_inner,
                 int64_t so, int64_t si, int64_t st, int32_t seqlen, int32_t nhead, int32_t dh,
                 int32_t dtype, void* stream);

/* MSDeformAttn default branch (ms_deform_attn.py:384-444) + ms_deform_attn_core_pytorch
 * (145-193): softmax of the attention logits over L*P, loc = ref + off/(W_l,H_l),
 * bilinear (zeros, align_corners=False) gather from the head-major memory, weighted sum.
 *  value:  [batch][S][nhead*dh] dtype; level l occupies rows [lvl_start[l], +h*w)
 *  offattn:[batch*lq][nhead*L*P*3] dtype: offsets (h,l,p,xy) then logits (h,l,p)
 *  ref:    [batch*lq][2] f32 (x, y) in [0,1];  out: [batch*lq] rows of ld_out, dtype */
enum { DP_MSDA_OFFATTN_F32 = 0x100 };  /* or'ed into dp_msda's dtype: offattn is f32 (training op) */
int dp_msda(const void* value, int32_t batch, int32_t S, const int32_t* lvl_hw /* [L][2] host */,
            int32_t nlevels, const void* offattn, const float* ref, void* out, int32_t ld_out,
            int32_t lq, int32_t nhead, int32_t dh, int32_t npoints, int32_t dtype, void* stream);

/* MSDA core at the training interface (explicit sampling locations and softmaxed attention
 * weights): ms_deform_attn_core_pytorch (ms_deform_attn.py:145-193) forward, and its autograd
 * (grid_sample bilinear/zeros/align_corners=False backward + weighted sum) for the training
 * step. value [N][S][nH*Dh] (dtype), loc f32 [N][Lq][nH][L][P][2], attn f32 [N][Lq][nH][L][P],
 * out / grad_out [N][Lq][nH*Dh] (dtype). Backward writes grad_value (f32, same shape as value;
 * cleared, then accumulated with atomics), grad_loc and grad_attn (f32, shapes of loc / attn).
 * The reference has no native MSDA op (CUDA-free build); these replace the autograd of the
 * pytorch core at the same call site (ms_deform_attn.py:436-441). */
int dp_msda_core_fwd(const void* value, int32_t batch, int32_t S, const int32_t* lvl_hw /* [L][2] host */,
                     int32_t nlevels, const float* loc, const float* attn, void* out, int32_t lq,
                     int32_t nhead, int32_t dh, int32_t npoints, int32_t dtype, void* stream);
int dp_msda_core_bwd(const void* value, int32_t batch, int32_t S, const int32_t* lvl_hw /* [L][2] host */,
                     int32_t nlevels, const float* loc, const float* attn, const void* grad_out,
                     int32_t lq, int32_t nhead, int32_t dh, int32_t npoints, float* grad_value,
                     float* grad_loc, float* grad_attn, int32_t dtype, void* stream);

/* Backward of dp_msda (MSDeformAttn.forward's default branch, ms_deform_attn.py:384-441,
 * the module-level training op): offattn f32 [batch*lq][nhead*L*P*2 | nhead*L*P] = the raw
 * sampling_offsets | attention_weights Linear outputs, ref f32 [batch*lq][2]. Recomputes the
 * softmax and the sampling locations and applies the chain rule through them in the same pass:
 * grad_value f32 (f32 atomics; zeroed here first unless accumulate_value) or NULL (value not
 * differentiated), grad_offattn f32 (offattn layout), grad_ref f32 [batch*lq][2] or NULL (zeroed
 * here; atomics over the heads). value / grad_out of dtype; grad_out rows ld_grad_out apart. */
int dp_msda_bwd(const void* value, int32_t batch, int32_t S, const int32_t* lvl_hw /* [L][2] host */,
                int32_t nlevels, const float* offattn, const float* ref, const void* grad_out, int32_t ld_grad_out,
                int32_t lq, int32_t nhead, int32_t dh, int32_t npoints, float* grad_value, int32_t accumulate_value,
                float* grad_offattn, float* grad_ref, int32_t dtype, void* stream);

/* dp_msda_bwd with the value gradient summed without float atomics (same arguments and
 * results; grad_value required, dh in {8, 16, 32, 64}): each sampling point is filed under the
 * top-left corner cell of its bilinear footprint by a per-(image, head, level) counting sort in
 * LDS, and each value pixel sums the lists of the four cells that cover it in registers, then
 * adds into grad_value once. workspace: device memory of dp_msda_bwd_ws_bytes(...) bytes
 * (reusable across calls on one stream); dp_msda_bwd_ws_bytes returns -1 for a shape the sort
 * cannot hold (a level's (H+1)(W+1) cells + lq*npoints points over 160 KiB of LDS). Same reference
 * interface as dp_msda_bwd (MSDeformAttn.forward's default branch backward,
 * ms_deform_attn.py:384-441 / ms_deform_attn_core_pytorch :145-193). */
int64_t dp_msda_bwd_ws_bytes(int32_t batch, int32_t S, const int32_t* lvl_hw /* [L][2] host */, int32_t nlevels,
                             int32_t lq, int32_t nhead, int32_t npoints);
int dp_msda_bwd_sorted(const void* value, int32_t batch, int32_t S, const int32_t* lvl_hw /* [L][2] host */,
                       int32_t nlevels, const float* offattn, const float* ref, const void* grad_out,
                       int32_t ld_grad_out, int32_t lq, int32_t nhead, int32_t dh, int32_t npoints,
                       float* grad_value, int32_t accumulate_value, float* grad_offattn, float* grad_ref,
                       void* workspace, int64_t workspace_bytes, int32_t dtype, void* stream);

/* Input pipeline of the reference benchmark (tools/benchmark/dataset.py:56-61) for one image
 * decoded to uint8 RGB (3, h, w) on the device: T.Resize to (new_h, new_w) (bilinear with
 * antialias, round + clamp to uint8, as torchvision's tensor resize), PadToSize(out_h, out_w)
 * with `fill` on the right / bottom, ConvertImageDtype(float) (/255) into out f32
 * (3, out_h, out_w), i.e. one slot of the model's input batch. The resize size is the
 * caller's (T.Resize(639, max_size=640) rule: detrpose_amd.preprocess.resized_size). */
int dp_resize_pad(const uint8_t* img, int32_t h, int32_t w, int32_t new_h, int32_t new_w,
                  float* out, int32_t out_h, int32_t out_w, float fill, void* stream);

/* dp_layernorm over contiguous rows (+ border mask) that also writes
 * cls_out[r] = max_j (y[r] . w[j] + b[j]), j < nclass, of the STORED (dtype-rounded) row y:
 * the two-stage enc_output_norm + enc_out_class_embed + .max(-1) (transformer.py:1232-1240)
 * in one pass (= dp_layernorm then dp_class_max, without re-reading the rows). */
int dp_layernorm_classmax(void* out, const void* x, const float* gamma, const float* beta, float eps,
                          int32_t rows, int32_t c, const uint8_t* row_mask, int32_t mask_period,
                          const float* masked_row, const float* cls_w, const float* cls_b, int32_t nclass,
                          float* cls_out, int32_t dtype, void* stream);

/* Per-row top-k of f32 scores, sorted descending, ties to the lower index:
 * torch.topk over the two-stage class score (transformer.py:1240) and in PostProcess
 * (postprocesses.py:19).  k <= 256, n <= 16384. idx is int64. */
int dp_topk(const float* x, int32_t rows, int32_t n, int32_t ld, int32_t k,
            float* out_val, int64_t* out_idx, void* stream);

/* out[r] = max_j (x[r] . w[j] + b[j]), j < nclass: enc_out_class_embed + .max(-1)
 * (transformer.py:1239-1240). w f32 [nclass][c]. */
int dp_class_max(const void* x, int32_t rows, int32_t c, const float* w, const float* b,
                 int32_t nclass, float* out, int32_t dtype, void* stream);

/* dst[b][j] = src[b][idx[b][j]] (rows of c elements): topk gather (transformer.py:1243-1248). */
int dp_gather_rows(const void* src, int64_t src_bstride, const int64_t* idx, int32_t batch, int32_t k,
                   int32_t c, void* dst, int32_t dtype, void* stream);

/* Two-stage reference points (transformer.py:1250-1254): kp = sigmoid(delta + anchor[idx]),
 * ref[b][q] = [mean(kp), kp...].  delta f32 [batch*k][nkp*2], anchors f32 [S][2]. */
int dp_refpoint_init(const float* delta, const float* anchors, const int64_t* idx, int32_t batch,
                     int32_t k, int32_t nkp, float* ref, void* stream);

/* Repeat a `bytes`-long block `count` times (query construction, transformer.py:1256-1261). */
int dp_broadcast(const void* src, int64_t bytes, void* dst, int32_t count, void* stream);

/* TransformerDecoder.sine_embedding of the keypoint refs (transformer.py:518-540):
 * ref f32 [rows][1+nkp][2] (centre skipped), dim_t f32 [c/2] (the decoder.dim_t buffer,
 * transformer.py:501-503) -> out [rows*nkp][c] dtype (pos_y | pos_x). */
int dp_sine_embed(const float* ref, int32_t rows, int32_t nkp, int32_t c, const float* dim_t,
                  void* out, int32_t dtype, void* stream);

/* Small-N linear in f32: out[r][n] = act(x[r] . w[:, n % nw] + b[n % nw]) + add[r][n]
 * (add optional), w f32 TRANSPOSED [k][nw].  x rows via row map, dtype x_dtype
 * (DP_F32 / DP_BF16); out rows contiguous [rows][n]. The f32 heads: pose / pre-pose /
 * class / LQE layers (transformer.py:705-728), enc_pose_embed last layer (1250). */
int dp_linear_small(const void* x, dp_rowmap xm, int32_t x_dtype, int32_t rows, int32_t k,
                    const float* w, const float* b, int32_t nw, int32_t n, int32_t act,
                    const float* add, float* out, void* stream);

/* Integral + distance2pose + centre (transformer.py:238-260, 198-219, 712-719):
 * corners f32 [rows*nkp][2*(reg_max+1)], project f32 [reg_max+1], ref_init f32
 * [rows*nkp][2] -> kps f32 [rows][nkp][2] and ref f32 [rows][1+nkp][2]. */
int dp_pose_refine(const float* corners, const float* project, int32_t reg_max, const float* ref_init,
                   float reg_scale, int32_t rows, int32_t nkp, float* kps, float* ref, void* stream);

/* pre_poses = sigmoid(pre + inverse_sigmoid(ref kp)) (transformer.py:705-709, utils.py:133-137). */
int dp_pre_pose(const float* pre, const float* ref, int32_t rows, int32_t nkp, float* out, void* stream);

/* LQE statistics (transformer.py:275-285): bilinear sample of feat (NHWC dtype, h x w x c)
 * at each keypoint, top-4 over channels + their mean -> out f32 [batch*nq][nkp*5]. */
int dp_lqe_stats(const void* feat, int64_t feat_bstride, int32_t h, int32_t w, int32_t c,
                 const float* kps, int32_t batch, int32_t nq, int32_t nkp, float* out,
                 int32_t dtype, void* stream);

/* PostProcess deploy branch (postprocesses.py:15-30), any batch. */
int dp_postprocess(const float* logits, const float* kps, const float* target_sizes, int32_t batch,
                   int32_t nq, int32_t nclass, int32_t nkp, int32_t num_select,
                   float* scores, int64_t* labels, float* out_kps, void* stream);

/* ---- Row-block fused decoder-layer kernels (bf16 only; c = hidden dim 128 / 256 / 384).
 * A block owns 64 token rows and all c channels, so the row-wise op after each GEMM runs
 * in its epilogue. Weights bf16 [n][k] (nn.Linear layout), biases f32. */

/* enc_output Linear + LayerNorm + masked rows + class-score max of the two-stage selection
 * (transformer.py:1232-1240) in one pass: out = LN(x . w^T + b) (rows with
 * row_mask[r % mask_period] != 0 take masked_row), cls_out[r] = max_j (out[r] . cls_w[j] +
 * cls_b[j]) over the stored bf16 row. bf16, contiguous rows of c = 256, w in the fragment
 * layout; replaces the enc_output dp_conv2d + dp_layernorm_classmax pair. */
int dp_linear_layernorm_classmax(void* out, const void* x, int32_t rows, int32_t c, const void* w, const float* b,
                                 const float* gamma, const float* beta, float eps, const uint8_t* row_mask,
                                 int32_t mask_period, const float* masked_row, const float* cls_w,
                                 const float* cls_b, int32_t nclass, float* cls_out, void* stream);

/* The whole token self-attention block of the decoder layer in one launch:
 * out = LayerNorm(x + MHA(x, x, x) . wo^T + bo) (+ post as dp_linear_layernorm), with
 * MHA = nn.MultiheadAttention(C, nhead) (in_proj wqkv [3C][C] + bqkv, out_proj wo [C][C] + bo,
 * both in the fragment layout). Replaces within_attn + within_norm and across_attn +
 * across_norm + the second in-place pos add (transformer.py:403-422). Token t of sequence
 * (o, ii) (o < n_outer, ii < n_inner, t < seqlen) is row o*so + ii*si + t*st of x and out.
 * C = 256 with 8 heads; seqlen 18 (within: the 1 + 17 tokens of a query) or 60 (across:
 * the queries of a token slot). out may not alias x. With next_out: also
 * next_out[r] = out[r] . next_w^T + next_b (next_n outputs, fragment layout) from the stored
 * rows -- the MSDA sampling-offset / attention-logit projection of the across attention's
 * output (ms_deform_attn.py:428-432). */
int dp_mha_layernorm(void* out, dp_rowmap om, const void* x, dp_rowmap xm, int32_t n_outer, int32_t n_inner,
                     int64_t so, int64_t si, int64_t st, int32_t seqlen, const void* wqkv, const float* bqkv,
                     const void* wo, const float* bo, const float* gamma, const float* beta, float eps, int32_t c,
                     int32_t nhead, const void* post, dp_rowmap pm, int32_t post_group, int32_t post_skip,
                     void* next_out, int32_t next_ld, const void* next_w, const float* next_b, int32_t next_n,
                     void* stream);

/* out = LayerNorm(x . w^T + b + res) (+ post on the rows the post map selects, as in
 * dp_layernorm). MultiheadAttention.out_proj + residual + LayerNorm of the decoder layer:
 * within_attn -> within_norm, across_attn -> across_norm + the second in-place pos add
 * (transformer.py:403-422, 360-370). k == c. out may not alias x. */
int dp_linear_layernorm(void* out, dp_rowmap om, const void* x, dp_rowmap xm, int32_t k,
                        const void* w, const float* b, const void* res, dp_rowmap rm,
                        const float* gamma, const float* beta, float eps, int32_t rows, int32_t c,
                        const void* post, dp_rowmap pm, int32_t post_group, int32_t post_skip,
                        void* stream);

/* Gate.forward (transformer.py:222-235) including its Linear: xcat rows [x1 | x2] (2c),
 * w [2c][2c]; out = LayerNorm(sigmoid(g1) * x1 + sigmoid(g2) * x2). */
int dp_gate_linear_layernorm(void* out, dp_rowmap om, const void* xcat, dp_rowmap xm,
                             const void* w, const float* b, const float* gamma, const float* beta,
                             float eps, int32_t rows, int32_t c, void* stream);

/* forward_ffn (transformer.py:371-385): out = LayerNorm(x + w2 . relu(w1 . x + b1) + b2),
 * w1 [f][c], w2 [c][f]; the hidden activations never leave the block. out may alias x. */
int dp_ffn_layernorm(void* out, dp_rowmap om, const void* x, dp_rowmap xm, const void* w1,
                     const float* b1, int32_t f, const void* w2, const float* b2,
                     const float* gamma, const float* beta, float eps, int32_t rows, int32_t c,
                     void* stream);

/* Query position of the keypoint tokens: sine_embedding of the keypoint reference points
 * (transformer.py:518-540) -> half_pose_ref_point_head MLP(c, c, c, 2) (588-592) ->
 * pos [rows][c], and the in-place with_pos_embed of the layer input (360-370):
 * tgt keypoint row r += pos[r]. rows = nq_rows * nkp keypoint tokens; ref f32
 * [nq_rows][nkp + 1][2] (row 0 of a query = its centre). */
int dp_query_pos(const float* ref, int32_t rows, int32_t nkp, const float* dim_t,
                 const void* w0, const float* b0, const void* w1, const float* b1,
                 void* pos, void* tgt, dp_rowmap tm, int32_t c, void* stream);

/* pose_embed[l] MLP(c, c, nout, 3) (utils.py:75-87) on x (+ x2, the reference's
 * output_pose + output_pose_detach) (+ prev: pred_corners + pred_corners_undetach):
 * transformer.py:705-719. out f32 [rows][nout], nout <= 128. */
int dp_pose_mlp(const void* x, dp_rowmap xm, const void* x2, dp_rowmap x2m, int32_t rows,
                const void* w0, const float* b0, const void* w1, const float* b1,
                const void* w2, const float* b2, int32_t nout, const float* prev, float* out,
                int32_t c, void* stream);

/* ---- Training criterion: matching + the default losses of the L/N/X
 * configs (criterion losses ['vfl', 'keypoints'], configs/detrpose/include/detrpose_hgnetv2.py).
 * Heads are the decoder outputs the reference matches: final, aux 0..L-2, pre, interm.
 * Targets are packed per batch: tgt_off [B+1] prefix offsets (int32), tgt_label [T] (int32),
 * tgt_kps [T][3K] f32 = K (x, y) pairs then K visibilities, tgt_area [T] f32. */

/* HungarianMatcher.forward (src/models/detrpose/matcher.py:47-112) for H heads at once:
 * logits (H, B, Q, ncls) and keypoints (H, B, Q, 2K) f32 at the given element strides;
 * cost = cost_class * focal + cost_kp * L1 + cost_oks * (1 - OKS) per image, solved by
 * scipy's shortest augmenting path (linear_sum_assignment, matcher.py:97) in f64 on the
 * GPU. match (H, B, Q) int32 = the image-local target index of query q, or -1; -2 for every
 * query of an image whose cost block is infeasible (NaN / inf costs, where scipy raises):
 * dp_pose_loss then returns a NaN loss_vfl for that head. The reference drops the keypoint
 * costs when a head's keypoints sum to <= 0 (matcher.py:70); sigmoid / refined keypoints
 * never do, so that branch is not built (the keypoint costs are always added).
 * max_t = the most targets of any image (LDS sizing). cost_out (H, B, Q, max_t) or NULL. */
int dp_hungarian_match(const float* logits, int64_t lg_h, int64_t lg_b, int32_t lg_q, int32_t ncls,
                       const float* kps, int64_t kp_h, int64_t kp_b, int32_t kp_q, int32_t nkp,
                       const int32_t* tgt_off, const int32_t* tgt_label, const float* tgt_kps,
                       const float* tgt_area, int32_t H, int32_t B, int32_t Q, int32_t max_t,
                       float cost_class, float cost_kp, float cost_oks, float alpha,
                       const float* sigmas, int32_t* match, float* cost_out, void* stream);

/* Criterion._get_go_indices (criterion.py:247-268): go (B, Q) = per query the target the
 * most of the H matchings chose (ties: the smallest target index), -1 if none;
 * n_go = number of matched queries (f32 scalar, before the all-reduce of criterion.py:306-312). */
int dp_match_union(const int32_t* match, int32_t H, int32_t B, int32_t Q, int32_t* go, float* n_go,
                   void* stream);

#define DP_LOSS_MAX_HEADS 16
/* One decoder head for dp_pose_loss: its logits (B, Q, ncls) and keypoints (B, Q, 2K) f32
 * at element strides, and its own matching (B, Q) from dp_hungarian_match. */
typedef struct dp_loss_head {
  const float* logits;  int64_t lg_b;  int32_t lg_q;
  const float* kps;     int64_t kp_b;  int32_t kp_q;
  const int32_t* match;
} dp_loss_head;

/* Criterion.loss_vfl (criterion.py:58-93) with the head's matching and loss_keypoints
 * (criterion.py:200-229: L1 + OKS, keypoint_loss.py) with the union matching go, for H heads:
 * losses (H, 3) = [loss_vfl * w_vfl, loss_keypoints * w_kp, loss_oks * w_oks], normalised by
 * max(n_boxes / world, 1) and max(n_boxes_go / world, 1) (device scalars, all-reduced by the
 * caller); and the gradients of those three weighted losses: g_logits (H, B, Q, ncls) of
 * loss_vfl, g_kp_l1 / g_kp_oks (H, B, Q, 2K) of loss_keypoints / loss_oks. */
int dp_pose_loss(const dp_loss_head* heads /* host array of H */, int32_t H, int32_t B, int32_t Q,
                 int32_t ncls, int32_t nkp, const int32_t* go, const int32_t* tgt_off,
                 const int32_t* tgt_label, const float* tgt_kps, const float* tgt_area,
                 const float* sigmas, float alpha, float gamma, const float* n_boxes,
                 const float* n_boxes_go, float world, float w_vfl, float w_kp, float w_oks,
                 float* losses, float* g_logits, float* g_kp_l1, float* g_kp_oks, void* stream);

/* ---- Training step (BASELINE config 5): the transformer's training forward
 * with OKS-denoising queries and its backward. Every nn.Linear forward / input gradient / weight
 * gradient is a dp_gemm; the row ops have explicit forward (saving what the backward needs) and
 * backward entry points. Activations and activation gradients are of `dtype`, LayerNorm
 * statistics, parameter gradients and head tensors f32. Callers: detrpose_amd/train_engine.py. */

/* C(b,m,n) = act(alpha * sum_k A(b,m,k) B(b,k,n) + bias[n] + beta * C(b,m,n)) (act: none / ReLU / GELU
 * (erf)), then zeroed where
 * gate(b,m,n) <= 0 (ReLU backward); A(b,m,k) = a[b*a_bs + m*a_rs + k*a_ks], B(b,k,n) =
 * b[b*b_bs + k*b_ks + n*b_ns], C(b,m,n) = c[b*c_bs + m*c_rs + n]. A and B of in_dtype, C of
 * out_dtype, f32 accumulation on MFMA. split_k 0 = automatic: a launch whose M x N grid cannot
 * fill the chip (weight gradients) splits K and accumulates into f32 C with atomics (needs
 * beta 1 and no bias / act / gate: C holds the initial value). Replaces nn.Linear and its
 * autograd (F.linear's addmm / mm backward). */
typedef struct dp_gemm_desc {
  const void* a; int64_t a_bs, a_rs, a_ks;
  const void* b; int64_t b_bs, b_ks, b_ns;
  void* c;       int64_t c_bs, c_rs;
  int32_t batch, m, n, k;
  int32_t in_dtype, out_dtype;
  const float* bias;
  float alpha, beta;
  int32_t act;
  const void* gate; int64_t gate_bs, gate_rs; int32_t gate_dtype;
  int32_t split_k;
  /* optional (NULL: none): colsum[m] += alpha * sum_k A(0, m, k) -- a Linear's bias gradient
   * (the column sums of dy) from the weight-gradient GEMM dW += dy^T x that already streams dy;
   * batch 1 */
  float* colsum;
} dp_gemm_desc;
int dp_gemm(const dp_gemm_desc* d, void* stream);

/* Weight gradient of a dense k x k conv without im2col columns (the training step's 3x3 convs:
 * ConvNormLayer / VGGBlock, hybrid_encoder.py:56-127; HG_Block's ConvBNAct, hgnetv2.py:82-134):
 * dw[cout][cin][kh][kw] += sum over output pixels p of dz[p][co] * x[tap's input pixel of p][ci]
 * (the reference weight layout). The 128 x 128 MFMA GEMM with its B tile gathered from NHWC x per
 * (pixel, tap, 8 channels) on the fly (zero outside the map), split-K f32 sums into scratch
 * [cout][kh*kw*cin] (zeroed here), then permuted into dw. x: batch images of h x w pixels
 * x_pstride apart (x_bstride per image), cin % 8 == 0; dz: batch*oh*ow rows dz_ld apart
 * (cout used). bf16 only. */
int dp_conv_wgrad(const void* x, int64_t x_bstride, int32_t x_pstride, int32_t batch, int32_t h, int32_t w,
                  int32_t cin, const void* dz, int64_t dz_ld, int32_t oh, int32_t ow, int32_t cout, int32_t kh,
                  int32_t kw, int32_t stride, int32_t pad, float* scratch, float* dw, int32_t dtype, void* stream);
/* dp_conv_wgrad on a scratch that holds zeros on entry and is left zeroed on return (the permute
 * clears each element it consumes), so no zero-fill launch per call: a training plan allocates each
 * conv's scratch zeroed once (torch.zeros). Same arguments and result. */
int dp_conv_wgrad_zs(const void* x, int64_t x_bstride, int32_t x_pstride, int32_t batch, int32_t h, int32_t w,
                     int32_t cin, const void* dz, int64_t dz_ld, int32_t oh, int32_t ow, int32_t cout, int32_t kh,
                     int32_t kw, int32_t stride, int32_t pad, float* scratch, float* dw, int32_t dtype, void* stream);

/* y = LayerNorm(x [+ res]) over contiguous rows of c (nn.LayerNorm, eps): writes y, the pre-norm
 * sum s = x + res (if s != NULL; the backward's input) and stats f32 [rows][2] = (mean, rstd);
 * x / res / s rows contiguous, y rows ld_y apart.
 * With post != NULL also y[r] += post[...] on the rows selected as in dp_layernorm (group /
 * skip: row r of a group of `post_group` rows takes post row (r / group) * (group - skip) +
 * (r % group - skip) when r % group >= skip): the decoder's second in-place pos add. */
int dp_ln_fwd(void* y, int32_t ld_y, const void* x, const void* res, void* s, float* stats, const float* gamma,
              const float* beta, float eps, int32_t rows, int32_t c, const void* post, int32_t post_group,
              int32_t post_skip, int32_t dtype, void* stream);
/* LayerNorm backward from the saved pre-norm input s and stats: dx (= or += when accumulate),
 * dgamma / dbeta f32 [c] accumulated (+=, the caller zeroes them once per step). */
int dp_ln_bwd(void* dx, const void* dy, int32_t ld_dy, const void* s, const float* stats, const float* gamma,
              int32_t rows, int32_t c, float* dgamma, float* dbeta, int32_t accumulate, int32_t dtype, void* stream);

/* out[n] (+)= sum over rows of x[r][n] (f32 out): bias gradients. x rows ld apart, of dtype. */
int dp_colsum(const void* x, int64_t ld, int32_t rows, int32_t n, float* out, int32_t accumulate, int32_t dtype,
              void* stream);

/* Softmax attention core for the training step, with an optional bool mask (mask[i*seqlen + j]
 * != 0: query i may not see key j; nn.MultiheadAttention attn_mask semantics). Sequences and
 * rows addressed as dp_attention (row o*so + i*si + t*st; q / k / v columns h*dh of rows ld_q /
 * ld_kv apart, out ld_o). Saves P f32 [seq][head][key][query] (softmax probabilities) for the
 * backward. dh 16 / 32 / 48 / 64; one wave per (sequence, head, 64 queries), keys streamed through LDS in
 * 64-row chunks (the decoder's 18 / 60 + DN tokens, the AIFI layer's 400: hybrid_encoder.py:276-279). */
int dp_attn_fwd(const void* q, int32_t ld_q, const void* k, const void* v, int32_t ld_kv, void* out, int32_t ld_o,
                float* p_save, const uint8_t* mask, int32_t n_outer, int32_t n_inner, int64_t so, int64_t si,
                int64_t st, int32_t seqlen, int32_t nhead, int32_t dh, int32_t dtype, void* stream);
/* Its backward: dq / dk / dv (same addressing as q / k / v, ld_dq / ld_dkv) from dout and the
 * forward's output out (both ld_o; D_i = dout_i . out_i); p_save is only read (the backward can be
 * replayed on the same forward). */
int dp_attn_bwd(const void* q, int32_t ld_q, const void* k, const void* v, int32_t ld_kv, const float* p_save,
                const void* dout, const void* out, int32_t ld_o, void* dq, int32_t ld_dq, void* dk, void* dv, int32_t ld_dkv,
                int32_t n_outer, int32_t n_inner, int64_t so, int64_t si, int64_t st, int32_t seqlen,
                int32_t nhead, int32_t dh, int32_t dtype, void* stream);

/* Gate.forward after its Linear (transformer.py:231-235): g = sigmoid(G) saved [rows][2c],
 * z = g1 * x1 + g2 * x2 with xcat = [x1 | x2] rows of 2c. */
int dp_gate_fwd(const void* G, const void* xcat, void* g, void* z, int32_t rows, int32_t c, int32_t dtype,
                void* stream);
/* Its backward from dz: dG = dg * g (1 - g) (pre-sigmoid) and dxcat = [dz g1 | dz g2] (the
 * direct path; the Linear's dgrad is added by dp_gemm with beta 1). */
int dp_gate_bwd(const void* dz, const void* g, const void* xcat, void* dG, void* dxcat, int32_t rows, int32_t c,
                int32_t dtype, void* stream);

/* Query construction of the training forward (transformer.py:1253-1261, 1278; DN queries of
 * dn_component.py:132-153): tgt [B][pad + nq][1 + K][c] = DN slots [label_enc[dn_label] |
 * pose_enc] (zero rows where dn_label < 0), then the matching queries [instance | tgt_embed[q] +
 * keypoint_embedding]. Weights f32, tgt of dtype. */
int dp_query_build(const float* tgt_embed, const float* kp_embed, const float* inst_embed, const float* label_enc,
                   const float* pose_enc, const int32_t* dn_label, int32_t batch, int32_t pad, int32_t nq,
                   int32_t nkp, int32_t c, void* tgt, int32_t dtype, void* stream);
/* Its backward: gradients (+=, f32) of the five embedding tables from dtgt. */
int dp_query_build_bwd(const void* dtgt, const int32_t* dn_label, int32_t batch, int32_t pad, int32_t nq,
                       int32_t nkp, int32_t c, float* g_tgt_embed, float* g_kp_embed, float* g_inst_embed,
                       float* g_label_enc, int32_t n_label, float* g_pose_enc, int32_t dtype, void* stream);

/* Backward of dp_pose_refine's keypoint output (Integral softmax . project, distance2pose):
 * dcorners [rows*nkp][2*(reg_max+1)] f32 (= or += when accumulate) from dkps [rows][nkp][2]. */
int dp_pose_refine_bwd(const float* corners, const float* project, int32_t reg_max, float reg_scale,
                       const float* dkps, int32_t rows, int32_t nkp, float* dcorners, int32_t accumulate,
                       void* stream);
/* pre_poses = sigmoid(pre + inverse_sigmoid(ref)) backward: dpre = dout * out * (1 - out). Also the
 * two-stage keypoints sigmoid(delta + anchor) (transformer.py:1243): the same elementwise rule.
 * out / dout / din f32 with element strides. */
int dp_sigmoid_bwd(const float* out, const float* dout, float* din, int32_t rows, int32_t n, int64_t ld_out,
                   int64_t ld_dout, int64_t ld_din, void* stream);
/* LQE statistics backward (transformer.py:275-285): dkps (+=) [batch*nq][nkp][2] from
 * dstats [batch*nq][nkp*5] through the top-4 / mean and the bilinear sampling coordinates;
 * with dfeat != NULL also d feats[0] (+=, f32 atomics, NHWC rows of c, images dfeat_bstride
 * apart: F.grid_sample's input gradient at the selected channels), else feats[0] is detached. */
int dp_lqe_stats_bwd(const void* feat, int64_t feat_bstride, int32_t h, int32_t w, int32_t c, const float* kps,
                     const float* dstats, int32_t batch, int32_t nq, int32_t nkp, float* dkps, float* dfeat,
                     int64_t dfeat_bstride, int32_t dtype, void* stream);
/* dst[idx[b][j]] (+)= src[b][j] rows of c (scatter of gathered rows; idx unique per image):
 * the backward of dp_gather_rows (of dp_gather_rows_masked with row_mask: rows whose
 * row_mask[idx % mask_period] != 0 receive nothing, memory.masked_fill's gradient). src rows
 * ld_src apart, dst rows ld apart, f32 or dtype. */
int dp_scatter_rows(const void* src, int32_t ld_src, const int64_t* idx, const uint8_t* row_mask,
                    int32_t mask_period, int32_t batch, int32_t k, int32_t c, void* dst, int64_t dst_bstride,
                    int32_t ld_dst, int32_t accumulate, int32_t dtype, void* stream);
/* dst[b][j] = src[b][idx[b][j]] rows of c, zero where row_mask[idx % mask_period] != 0: the
 * masked memory rows the two-stage selection picked (memory.masked_fill(valid_mask, 0),
 * transformer.py:1221), for the enc_output backward on the selected rows only. */
int dp_gather_rows_masked(const void* src, int64_t src_bstride, const int64_t* idx, const uint8_t* row_mask,
                          int32_t mask_period, int32_t batch, int32_t k, int32_t c, void* dst, int32_t dtype,
                          void* stream);
/* prepare_for_cdn's random part (dn_component.py:51-153) on the device: for DN slot
 * group * single_pad + t (t < targets of the image; even groups positive, odd negative) the
 * target's label, replaced with probability label_noise_ratio / 2 by a uniform class <
 * num_classes, and its 1 + K points (xyxy-box centre, keypoints) with visible keypoints moved
 * along a first-quadrant unit direction by sqrt(alpha * 2 (area h w + eps) (2 sigma)^2) / max(h, w),
 * alpha ~ U(0, ln 2) (positive) / U(ln 2, ln 10) (negative); out dn_label [B][pad] (-1 padding)
 * and dn_ref [B][pad][1+K][2] = sigmoid(inverse_sigmoid(point)) (0.5 padding). sigmas [1+K]
 * (0.1 for the centre, then the keypoint sigmas). Counter-based RNG (seed): the draws are
 * distributed as the reference's torch.rand draws, not the same numbers. */
int dp_cdn_build(const int32_t* tgt_off, const int32_t* tgt_label, const float* tgt_kps, const float* tgt_area,
                 const float* tgt_boxes, const float* sigmas, int32_t batch, int32_t pad, int32_t single_pad,
                 int32_t nkp, float label_noise_ratio, int32_t num_classes, float img_h, float img_w, uint64_t seed,
                 int32_t* dn_label, float* dn_ref, void* stream);
/* Squared L2 norm of a gradient buffer: clip_grad_norm_'s norm, into out[0]. ws receives the
 * block partials: it must hold dp_grad_sqnorm_ws_floats(n) floats (at most DP_SQNORM_PARTS;
 * checked, an error otherwise). Deterministic (fixed-order reduction, no float atomics):
 * identical gradients give bit-identical norms on every rank. */
#define DP_SQNORM_PARTS 1024
int64_t dp_grad_sqnorm_ws_floats(int64_t n);
int dp_grad_sqnorm(const float* g, int64_t n, float* out, float* ws, int64_t ws_floats, void* stream);
/* torch.optim.AdamW step over a flat f32 parameter buffer (decoupled weight decay, bias
 * correction for `step`), after clip_grad_norm_(max_norm) (src/solver/engine.py:78-89) read
 * from grad_sqnorm on the device (max_norm <= 0: no clipping). Parameters and moments are left
 * unchanged when *skip != 0 (skip may be NULL) or the norm is not finite: the reference stops
 * before optimizer.step on a non-finite loss (engine.py:62-66). */
int dp_adamw(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float lr, float beta1,
             float beta2, float eps, float weight_decay, int32_t step, float max_norm, const float* grad_sqnorm,
             const float* skip, void* stream);
/* *bad = 1 when any of v[0..n) is not finite (unchanged otherwise): the step guard dp_adamw /
 * dp_ema read (engine.py:62-66's math.isfinite(loss) check, on the device). */
int dp_finite_guard(const float* v, int64_t n, float* bad, void* stream);
/* ModelEMA.update over a flat f32 buffer (src/nn/optimizer/ema.py:55-70): ema = decay ema +
 * (1 - decay) p, skipped when *skip != 0 (skip may be NULL). */
int dp_ema(float* ema, const float* p, int64_t n, float decay, const float* skip, void* stream);
/* hipMemsetAsync(p, 0, bytes) on the stream (gradient buffers at the start of a step). */
int dp_zero(void* p, int64_t bytes, void* stream);
/* Element conversion / copy between f32 and dtype rows (the head outputs' f32 views, gradient
 * hand-offs): dst[r][j] = src[r][j] (+ dst when accumulate) * scale. */
int dp_convert_rows(const void* src, int32_t src_dtype, int64_t ld_src, void* dst, int32_t dst_dtype,
                    int64_t ld_dst, int32_t rows, int32_t n, float scale, int32_t accumulate, void* stream);
/* A table of f32 row copies in ONE launch: dst[r][j] = src0[r][j] (+ src1[r][j] when src1 is not
 * NULL) for r < rows, j < n, each operand at its own row pitch (elements). The criterion's head
 * packing and gradient hand-off (criterion.py:285-435's outputs -> loss inputs, loss gradients ->
 * head-output gradients), which were one dp_convert_rows each. Entries must not write what
 * another entry reads or writes. dp_copy_rows_check validates a host copy of the table (once,
 * when it is built); dp_copy_rows_batch reads it from device memory (tab_dev), blocks_per_entry
 * blocks striding over each entry's elements. */
typedef struct dp_rowcopy_desc {
  const float* src0;
  const float* src1;
  float* dst;
  int64_t ld_src0, ld_src1, ld_dst;
  int32_t rows, n;
} dp_rowcopy_desc;
int dp_copy_rows_check(const dp_rowcopy_desc* tab, int32_t n);
int dp_copy_rows_batch(const dp_rowcopy_desc* tab_dev, int32_t n, int32_t blocks_per_entry, void* stream);

/* ---- HybridEncoder training step (BASELINE config 5; hybrid_encoder.py:56-212, 246-296,
 * 462-507 in training mode). Activations are NHWC rows [rows = batch*h*w][c] with a row stride
 * (ld, elements: channel slices of concat buffers), of dtype; statistics / parameter gradients
 * f32. Callers: detrpose_amd/encoder_train.py. */

/* nn.BatchNorm2d batch statistics, per rank: out [3][c] = (K = x[0][ch], sum (x - K), sum (x - K)^2)
 * over the rows (single pass, shifted by the first row against cancellation). Per-row-slice
 * partial sums go to ws (dp_bn_stats_ws_bytes) and are added in a fixed order: no float
 * atomics, the same result on every run. */
int64_t dp_bn_stats_ws_bytes(int32_t rows, int32_t c);
int dp_bn_stats(const void* x, int64_t ld, int32_t rows, int32_t c, float* out, float* ws, int64_t ws_bytes,
                int32_t dtype, void* stream);
/* Combines nparts per-rank dp_bn_stats outputs (all-gathered: SyncBatchNorm, dist_utils.py:122;
 * `count` rows each) into mean_rstd [2][c] = (mean, 1/sqrt(biased var + eps)) and updates the
 * running statistics as F.batch_norm does (momentum, unbiased variance; NULL: no update). */
int dp_bn_finalize(const float* parts, int32_t nparts, float count, int32_t c, float eps, float momentum,
                   float* running_mean, float* running_var, float* mean_rstd, void* stream);
/* dp_bn_stats then dp_bn_finalize of its single part (nparts 1, count = rows) in the statistics'
 * launches: BatchNorm on one rank, no SyncBN exchange between the two. Same arithmetic, so the
 * same outputs (out, mean_rstd, running statistics) bit for bit. */
int dp_bn_stats_finalize(const void* x, int64_t ld, int32_t rows, int32_t c, float* out, float* ws, int64_t ws_bytes,
                         float eps, float momentum, float* running_mean, float* running_var, float* mean_rstd,
                         int32_t dtype, void* stream);
/* y = act(g1 (z1 - mean1) rstd1 + b1 [+ g2 (z2 - mean2) rstd2 + b2]) [+ res]: ConvNormLayer's
 * norm + act (one branch) and VGGBlock's act(BN(conv3x3) + BN(conv1x1)) (two branches); res is
 * the CSP sum's other operand when fused. act: DP_ACT_*. */
int dp_bn_act_fwd(void* y, int64_t ld_y, const void* z1, int64_t ld1, const float* mr1, const float* g1,
                  const float* b1, const void* z2, int64_t ld2, const float* mr2, const float* g2, const float* b2,
                  const void* res, int64_t ld_res, int32_t rows, int32_t c, int32_t act, int32_t dtype, void* stream);
/* Its backward, first pass: dp = dy * act'(pre) (pre recomputed from z / statistics); sums [3][c] =
 * (sum dp, sum dp xhat1, sum dp xhat2) over this rank's rows (overwritten; all-reduce them for
 * SyncBN before the second pass) and, from the LOCAL sums, dg_k += sum dp xhat_k, db_k += sum dp
 * (NULL to skip). Per-256-row partials in ws (dp_bn_act_bwd_reduce_ws_bytes), summed in a fixed
 * order: the same result on every run. */
int dp_bn_act_bwd_reduce(const void* dy, int64_t ld_dy, const void* z1, int64_t ld1, const float* mr1,
                         const float* g1, const float* b1, const void* z2, int64_t ld2, const float* mr2,
                         const float* g2, const float* b2, int32_t rows, int32_t c, int32_t act, float* sums,
                         float* dg1, float* db1, float* dg2, float* db2, float* ws, int64_t ws_bytes, int32_t dtype,
                         void* stream);
/* Per-256-row-slice partials of dp_bn_act_bwd_reduce (summed in a fixed order: no float atomics). */
int64_t dp_bn_act_bwd_reduce_ws_bytes(int32_t rows, int32_t c);
/* Second pass: dz_k = g_k rstd_k (dp - sum dp / count - xhat_k sum (dp xhat_k) / count), count =
 * the rows of all ranks (batch_norm_backward_elemt). */
int dp_bn_act_bwd_apply(void* dz1, int64_t ld_dz1, void* dz2, int64_t ld_dz2, const void* dy, int64_t ld_dy,
                        const void* z1, int64_t ld1, const float* mr1, const float* g1, const float* b1,
                        const void* z2, int64_t ld2, const float* mr2, const float* g2, const float* b2,
                        int32_t rows, int32_t c, int32_t act, const float* sums, float count, int32_t dtype,
                        void* stream);
/* col [batch*oh*ow][cin*kh*kw] (of dtype) = the conv's input patches, K order (cin, ky, kx): dp_gemm
 * of dz^T with it is the weight gradient in the reference layout [cout][cin][kh][kw]. x of x_dtype,
 * element (b, y, x, c) at b*bstride + (y*w + x)*pstride + c*cstride (NHWC: cstride 1; the f32
 * NCHW image of stem1: pstride 1, cstride h*w). */
int dp_im2col(const void* x, int64_t bstride, int32_t pstride, int64_t cstride, int32_t batch, int32_t h, int32_t w,
              int32_t cin, int32_t kh, int32_t kw, int32_t stride, int32_t pad, int32_t oh, int32_t ow, void* col,
              int32_t x_dtype, int32_t dtype, void* stream);
/* f32 master conv weights [cout][cin][kh][kw] -> dp_conv2d's packed layout: mode 0 [cout][kpad]
 * (K = ky, kx, cin; the forward), mode 1 [cin][kpad] (K = ky, kx, cout, taps rotated by 180
 * degrees: the stride-1 input gradient as a conv of dz), mode 2 depthwise taps f32 [kh*kw][cout]
 * (cin = 1, dp_dwconv2d's layout), mode 3 f32 [cout][cin*kh*kw] (dp_stem_conv's layout), mode 4
 * [kh*kw*cin][kpad >= cout] (rows tap-major ky, kx, ci; K over cout: W^T for the column GEMM
 * dcol = dz W that dp_col2im reads). kc:
 * channel stride of K (the padded channel count of the map the packed conv reads, zero weights
 * in the pads; 0 = unpadded). scale (f32 [cout], NULL = 1): every output channel's weights
 * multiplied by it (FrozenBatchNorm2d's scale folded into the conv, hgnetv2.py:51-61). */
int dp_conv_pack(const float* w, int32_t cout, int32_t cin, int32_t kh, int32_t kw, void* out, int32_t kpad,
                 int32_t kc, int32_t mode, const float* scale, int32_t dtype, void* stream);
/* One dp_conv_pack call per entry (same fields; mode 5: a plain f32 -> dtype copy of `cout`
 * elements, the bf16 copy of a linear weight), all in ONE launch: a training plan's weight packs
 * of one optimizer step. dp_conv_pack_check validates a host copy of the table (once, when the
 * plan is built); dp_conv_pack_batch reads the table from device memory (tab_dev), its x blocks
 * striding over each pack's elements (blocks_per_pack of them). */
typedef struct dp_pack_desc {
  const float* w;
  void* out;
  const float* scale;
  int32_t cout, cin, kh, kw, kpad, kc, mode, dtype;
} dp_pack_desc;
int dp_conv_pack_check(const dp_pack_desc* tab, int32_t n);
int dp_conv_pack_batch(const dp_pack_desc* tab_dev, int32_t n, int32_t blocks_per_pack, void* stream);
/* Depthwise conv backward (k <= 5, any stride / pad): dx (+=, NULL to skip) and dw f32
 * [c][k][k] (+=, NULL to skip) from dz. x / dz / dx: NHWC with image and pixel strides. */
int dp_dwconv_bwd(const void* x, int64_t x_bstride, int32_t x_pstride, const void* dz, int64_t z_bstride,
                  int32_t z_pstride, const float* wt, int32_t batch, int32_t h, int32_t w, int32_t c, int32_t k,
                  int32_t stride, int32_t pad, int32_t oh, int32_t ow, void* dx, int64_t dx_bstride,
                  int32_t dx_pstride, float* dw, int32_t dtype, void* stream);
/* Nearest x2 upsample of an h x w map (F.interpolate(scale_factor=2.), hybrid_encoder.py:487):
 * backward == 0: dst (2h x 2w) = copy; backward != 0: src is the 2h x 2w gradient and dst
 * (h x w) += its 2x2 sums. */
int dp_upsample2x(const void* src, int64_t src_bstride, int32_t src_pstride, int32_t batch, int32_t h, int32_t w,
                  int32_t c, void* dst, int64_t dst_bstride, int32_t dst_pstride, int32_t backward, int32_t dtype,
                  void* stream);
/* y (= or +=) alpha a + beta b (b may be NULL): residual sums and gradient fan-out. */
int dp_axpby_rows(void* y, int64_t ld_y, const void* a, int64_t ld_a, float alpha, const void* b, int64_t ld_b,
                  float beta, int32_t rows, int32_t c, int32_t accumulate, int32_t dtype, void* stream);
/* dx = dy * act'(pre) (elementwise; the AIFI FFN's GELU backward). */
int dp_act_bwd(const void* pre, int64_t ld_pre, const void* dy, int64_t ld_dy, void* dx, int64_t ld_dx, int32_t rows,
               int32_t c, int32_t act, int32_t dtype, void* stream);


/* ---- HGNetv2 backbone training step (BASELINE config 5: freeze_at=-1 trains every backbone
 * parameter, freeze_norm=True keeps FrozenBatchNorm2d; hgnetv2.py:24-61, 82-383). Callers:
 * detrpose_amd/backbone_train.py. */

/* Backward of ConvBNAct's epilogue y = lab(act(s z + b)) [+ res] from its stored output
 * (hgnetv2.py:129-134; res: the HG block's identity added after it, hgnetv2.py:326-329, NULL =
 * none): dz = dy * a * act'(.) * scale[ch] (scale: the frozen BN scale, NULL = 1; a = *lab_a, or 1
 * without LAB); with the LAB scalars (device lab_a / lab_b, NULL = no LAB) *dlab_a += sum dy *
 * relu(.), *dlab_b += sum dy. act: DP_ACT_NONE (y unused) or DP_ACT_RELU. Rows ld apart, of dtype. */
int dp_frozen_act_bwd(const void* y, int64_t ld_y, const void* res, int64_t ld_res, const void* dy, int64_t ld_dy,
                      void* dz, int64_t ld_dz,
                      int32_t rows, int32_t c, int32_t act, const float* lab_a, const float* lab_b, const float* scale,
                      float* dlab_a, float* dlab_b, int32_t dtype, void* stream);
/* dx (= or += when accumulate) = col2im(col): col [batch*oh*ow][kh*kw*cin] (K order ky, kx, cin) =
 * dz W of a stride-s, pad-p conv; each input pixel sums the columns that read it (StemBlock.stem3's
 * 3x3 stride-2 input gradient). dx NHWC with image / pixel strides. */
int dp_col2im(const void* col, int32_t batch, int32_t h, int32_t w, int32_t cin, int32_t kh, int32_t kw,
              int32_t stride, int32_t pad, int32_t oh, int32_t ow, void* dx, int64_t dx_bstride, int32_t dx_pstride,
              int32_t accumulate, int32_t dtype, void* stream);
/* Backward of dp_maxpool2x2_pad_rb (F.pad(0,1,0,1) + MaxPool2d(2, 1, ceil_mode=True), hgnetv2.py:215,
 * 217): dx += each window's output gradient at the window's first maximum in scan order (the pad
 * zeros take part; a pad maximum drops the gradient). x: the pool's input. */
int dp_maxpool2x2_pad_rb_bwd(const void* x, int64_t x_bstride, int32_t x_pstride, const void* dout,
                             int64_t dout_bstride, int32_t dout_pstride, int32_t batch, int32_t h, int32_t w, int32_t c,
                             void* dx, int64_t dx_bstride, int32_t dx_pstride, int32_t dtype, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DETRPOSE_HIP_H */
