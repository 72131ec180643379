/*
 * vfd_capi.h — C ABI of the MI355X (gfx950) hot-path kernels of the VFDepth training step.
 *
 * The reference (tronglh241/VFDepth) is pure PyTorch: its hot path is a set of ATen calls
 * behind Python module APIs.  Each entry point below replaces the ATen call chain named in
 * its comment (paths relative to /root/reference).  Conventions:
 *   - all tensors are raw device pointers, fp32, contiguous in the layouts stated, allocated
 *     and owned by the caller (PyTorch's caching allocator); kernels never allocate;
 *   - `stream` is a hipStream_t (the caller's current stream); every call is asynchronous;
 *   - return 0 on success, a negative vfd_status on a bad descriptor or launch failure, with
 *     a message in vfd_last_error() (thread-local);
 *   - outputs the kernel accumulates into with atomics are zeroed inside the call;
 *   - "workspace" buffers are scratch of at least the *_workspace_bytes() size.
 * Layout symbols: B batch, N cameras, C feature channels, Cv voxel channels, (h, w) fusion-level
 * feature map, (H, W) image, (X, Y, Z) voxel counts, V = X*Y*Z (x fastest), D depth bins.
 */
#ifndef VFD_CAPI_H
#define VFD_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum vfd_status { VFD_OK = 0, VFD_EINVAL = -1, VFD_ELAUNCH = -2 };

int vfd_version(void);
const char* vfd_last_error(void);

/* ------------------------------------------------------------------ volumetric fusion */
typedef struct vfd_voxel_desc {
  int32_t B, N;          /* batch, cameras                                               */
  int32_t C;             /* image feature channels  (model.fusion_feat_in_dim)          */
  int32_t Cv;            /* voxel feature channels  (model.voxel_pre_dim[-1]), <= 128    */
  int32_t h, w;          /* feature map at the fusion level (H, W / 2^(fusion_level+1))  */
  int32_t H, W;          /* full-resolution mask                                         */
  int32_t X, Y, Z;       /* voxel counts (model.voxel_size)                              */
  int32_t D;             /* frustum depth bins (model.proj_d_bins)                       */
  float str[3];          /* model.voxel_str_p                                            */
  float len[3];          /* voxel_end_p - voxel_str_p                                    */
  float z_scale;         /* model.voxel_size[0]: divisor of the appended depth feature   */
  int32_t pad_out;       /* 1: outputs consumed by a 3x3 reflect conv are written padded;
                            2 (K3C only): padded layout, and the gradient of that padded map
                            arrives with its reflect copies already folded into the interior
                            (vfd_proj_conv_dgrad's folded form): the K3 plan / backward read every
                            sample from the interior, no fold pass */
  const float* axis_x;   /* [X] voxel centres (torch.linspace fp32), device              */
  const float* axis_y;   /* [Y]                                                          */
  const float* axis_z;   /* [Z]                                                          */
  const float* dbins;    /* [D] frustum depths (torch.linspace fp32), device             */
  const int32_t* group;  /* [N] overlap group of each camera (0: {0,3,4}, 1: {1,2,5})    */
  int32_t deterministic; /* 1: every gradient sums in a fixed order (torch.backends.cudnn.  */
                         /*    deterministic, as the reference's train.py:23 sets): the   */
                         /*    fusion plan's buckets and K3's cell lists are ordered by   */
                         /*    voxel / sample, and K3's heavy tiles are not split         */
} vfd_voxel_desc;

/* F.interpolate(mask, [h, w], 'bilinear', align_corners=True)
 * (network/volumetric_fusionnet.py:129).  mask [B*N, H, W] -> mask_lo [B*N, h, w]. */
int vfd_mask_downsample(const vfd_voxel_desc* d, const float* mask, float* mask_lo, void* stream);

/* K1 — depth-mode unprojection + overlap/non-overlap 1x1 MLP + LeakyReLU + masks
 * (volumetric_fusionnet.py:116-158, 166-230).  The 1x1 conv's feature columns are folded
 * into the per-camera maps by the caller: P[b,n,pix,0:Cv] = W_no[:, :C] f,
 * P[b,n,pix,Cv:2Cv] = W_o[:, g(n)(C+1) : g(n)(C+1)+C] f   (P: [B, N, h*w, 2*Cv]).
 * wz [3, Cv] = depth-feature columns (W_no[:,C], W_o[:,C], W_o[:,2C+1]); b_no, b_o [Cv].
 * K [B,N,4,4] at the fusion scale, Einv [B,N,4,4].  Output vox [B, V, Cv] (channels-last). */
int vfd_fuse_depth_fwd(const vfd_voxel_desc* d, const float* P, const float* mask_lo,
                       const float* K, const float* Einv, const float* wz, const float* b_no,
                       const float* b_o, float* vox, void* stream);
size_t vfd_fuse_depth_bwd_workspace(const vfd_voxel_desc* d);
/* d_vox [B,V,Cv], vox (forward output).  dP [B,N,h*w,2*Cv] (zeroed here);
 * d_wzb [5, Cv] = d wz (3 rows), d b_no, d b_o. */
int vfd_fuse_depth_bwd(const vfd_voxel_desc* d, const float* d_vox, const float* vox,
                       const float* mask_lo, const float* K, const float* Einv, float* dP,
                       float* d_wzb, void* workspace, size_t ws_bytes, void* stream);
/* K1 backward as an atomic-free gather over the fusion plan's tile buckets (the plan vfd_fusion_plan
 * builds for the K2 backward; same arguments otherwise, Cv = 64): d P written with plain stores,
 * summed in bucket order (deterministic once the buckets are, see vfd_fusion_plan_sort).  Its
 * workspace (vfd_fuse_depth_bwd_planned_workspace bytes) also holds its split tiles' partials, so
 * it may run concurrently with the K2 backward that reads the same plan (the pose branch's stream). */
size_t vfd_fuse_depth_bwd_planned_workspace(const vfd_voxel_desc* d);
int vfd_fuse_depth_bwd_planned(const vfd_voxel_desc* d, const void* plan, const float* d_vox, const float* vox,
                               const float* mask_lo, const float* K, const float* Einv, float* dP, float* d_wzb,
                               void* workspace, size_t ws_bytes, void* stream);

/* Fusion plan (volumetric_fusionnet.py:132-140, 166-195): for every (batch, camera) the compacted
 * list of voxels the camera sees (32-B entries: voxel | valid-camera count | in-range taps, corner
 * pixel, bilinear fractions, camera depth, mean denominator) and its length in counts [B*N],
 * plus its inverse index (per pixel, the (entry, tap) pairs that sample it; CSR).
 * Built once per step from K (fusion scale), Einv and mask_lo; shared by every pose-mode call. */
size_t vfd_fusion_plan_bytes(const vfd_voxel_desc* d);
int vfd_fusion_plan(const vfd_voxel_desc* d, const float* mask_lo, const float* K, const float* Einv,
                    void* plan, int* counts, void* stream);

/* K2 — pose-mode unprojection, mean over valid cameras (volumetric_fusionnet.py:116-162).
 * Voxel-major gather: every output element is written exactly once (no pre-zeroing, no atomics).
 * feats_cl [B,N,h*w,C] (channels-last), mask_lo [B*N,h,w], K / Einv [B,N,4,4] (fusion scale)
 * -> out [B, Y(+2), X(+2), Z*(C+1)]: NHWC input of reduce_dim's stride-2 3x3 conv (:339-342),
 * reflect-padded when pad_out, channel index z*(C+1) + c (the reference's c*Z + z order permuted;
 * the conv weight's input channels are permuted the same way, so the convolution is unchanged). */
int vfd_fuse_pose_fwd(const vfd_voxel_desc* d, const float* mask_lo, const float* K, const float* Einv,
                      const float* feats_cl, float* out, void* stream);
/* As vfd_fuse_pose_fwd with the map stored as dtype_out (0 fp32, 1 bf16 rounded to nearest even:
 * config 3, whose only consumer, the bf16 K2C, stages exactly those rounded values) and an
 * optional voxel order (nullable): [8][order_cap] voxel indices by azimuth sector around the rig,
 * -1 padding, every voxel exactly once; workgroup k takes sector k % 8, i.e. one XCD per sector
 * (its L2 then caches the features of the cameras facing it).  The output does not depend on it. */
int vfd_fuse_pose_fwd_t(const vfd_voxel_desc* d, const float* mask_lo, const float* K, const float* Einv,
                        const float* feats_cl, void* out, int dtype_out, const int* order, int order_cap,
                        void* stream);
/* d_out in the forward's output layout -> d_feats [B,N,C,h,w] (every element written).
 * Atomic-free gather over the plan's 4x4-pixel tile buckets, pulled from the plan's task queue
 * (heavy tiles split by channel group); the call resets the queue's work counter inside `plan`,
 * so calls sharing one plan must be stream-ordered. */
int vfd_fuse_pose_bwd(const vfd_voxel_desc* d, const void* plan, const int* counts, const float* d_out,
                      float* d_feats, void* stream);
/* the same with d_out of dtype_out (0 fp32, 1 bf16: the bf16 K2C data gradient, read 4 channels per
 * 8-B load and summed in fp32; the reflect copies are folded in fp32) */
int vfd_fuse_pose_bwd_t(const vfd_voxel_desc* d, const void* plan, const int* counts, const void* d_out,
                        int dtype_out, float* d_feats, void* stream);

/* K3 — voxel -> camera-frustum trilinear resampling (volumetric_fusionnet.py:232-262).
 * vox [B,V,Cv] (Cv <= 64), invK, E [B,N,4,4] (fusion scale) -> out [B*N, h(+2), w(+2), D*Cv]:
 * NHWC input of reduce_dim's first 3x3 conv, reflect-padded when pad_out, channel index
 * d*Cv + c (the reference's c*D + d order permuted; the conv weight is permuted to match). */
int vfd_voxel_project_fwd(const vfd_voxel_desc* d, const float* vox, const float* invK,
                          const float* E, float* out, void* stream);
/* Autograd of the trilinear gather (grid_sampler_3d_backward, volumetric_fusionnet.py:261-262):
 * d_out (forward layout, reflect copies folded) -> d_vox [B,V,Cv] (fully written here).
 * Two phases: (1) vfd_voxel_project_plan — geometry only (invK, E, depth bins): counting sort of
 * the frustum samples by voxel cell, tile parts, task list, into a device buffer of
 * vfd_voxel_project_plan_bytes(d) bytes; independent of d_out, so it can run on a side stream
 * while the forward's dense layers run; (2) vfd_voxel_project_bwd_planned — fold the reflect
 * copies of d_out and accumulate each voxel tile in LDS from the sorted samples.  A plan serves any
 * number of backward calls with the same descriptor / geometry.  vfd_voxel_project_bwd does both
 * in one call (workspace = the plan buffer).  No host sync; graph-safe. */
size_t vfd_voxel_project_plan_bytes(const vfd_voxel_desc* d);
int vfd_voxel_project_plan(const vfd_voxel_desc* d, const float* invK, const float* E, void* plan,
                           size_t plan_bytes, void* stream);
int vfd_voxel_project_bwd_planned(const vfd_voxel_desc* d, const float* d_out, void* plan,
                                  size_t plan_bytes, float* d_vox, void* stream);
size_t vfd_voxel_project_bwd_workspace(const vfd_voxel_desc* d);
int vfd_voxel_project_bwd(const vfd_voxel_desc* d, const float* d_out, const float* invK,
                          const float* E, float* d_vox, void* ws, size_t ws_bytes, void* stream);

/* K3C — K3 fused into reduce_dim's first 3x3 conv (volumetric_fusionnet.py:59-60, 232-267; depth
 * mode): out = LeakyReLU_0.1(conv3x3_reflect(frustum samples of vox) + bias) as an fp32 MFMA
 * implicit GEMM; the [B*N, Cv*D, h, w] frustum features are generated per (pixel tile, depth bin)
 * in LDS and never written.  vox [B,V,Cv] (Cv = 64), invK, E [B,N,4,4] (fusion scale),
 * Wq = the conv weight [O, Cv*D, 3, 3] in fragment order [D, 3, 3, Cv/4, O, 2, 2]
 * (reference channel c*D + d with c = 4q + 2h + s), bias [O], out_channels O = 256 ->
 * out [B*N, h+2, w+2, O]: reflect-padded NHWC input of reduce_dim's second conv.  D <= 64.
 * x_out (nullable): also write the frustum features themselves as [B*N, h+2, w+2, D*Cv] (channel
 * d*Cv + c, reflect-padded NHWC: K3's padded output layout) for the conv's backward.
 * Workspace: per-workgroup partial tiles (summed in a fixed order: deterministic). */
size_t vfd_proj_conv_fwd_workspace(const vfd_voxel_desc* d);
int vfd_proj_conv_fwd(const vfd_voxel_desc* d, const float* vox, const float* invK, const float* E,
                      const float* Wq, const float* bias, int out_channels, float* out, float* x_out,
                      void* workspace, size_t ws_bytes, void* stream);
/* bf16 form (config 3's autocast, volumetric_fusionnet.py:105-114): the same computation with the
 * halo samples rounded to bf16 and bf16 weights on v_mfma_f32_32x32x16_bf16 (fp32 accumulation,
 * bias and LeakyReLU in fp32).  vox / invK / E / bias fp32; Wq = vfd_weight_fragments_bf16 mode 3;
 * out and x_out (nullable) bf16, same layouts as vfd_proj_conv_fwd; same workspace size. */
int vfd_proj_conv_fwd_bf16(const vfd_voxel_desc* d, const float* vox, const float* invK, const float* E,
                           const void* Wq, const float* bias, int out_channels, void* out, void* x_out,
                           void* workspace, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------ fused BatchNorm (+res)(+ReLU) */
/* Training-mode BatchNorm2d of the ResNet encoders (fusion_depthnet.py:24-36, fusion_posenet.py:
 * 22-35; torchvision BasicBlock/Bottleneck/stem), fused with the block's residual add and ReLU:
 * y = relu((x - mean) * invstd * gamma + beta [+ r]), NCHW fp32.  Statistics in fp64, per
 * (channel, split) partials [C][S][2] summed in a fixed order.  SyncBatchNorm (DDP,
 * models/vfdepth.py:68 convert_sync_batchnorm): vfd_bn_sum reduces the partials to [C+1][2] sums
 * whose row C carries the local element count; the host all-reduces that buffer (ONE collective per
 * direction, like torch's SyncBatchNorm: one all_gather forward, one all_reduce backward) and the
 * apply passes take ns = 1 and count = 0, which makes them read the global count from row C on the
 * device (no host synchronisation). */
typedef struct vfd_bn_desc {
  int32_t N, C, HW;      /* images, channels, H*W                                        */
  int32_t S;             /* splits per channel: vfd_bn_splits(desc)                      */
  int32_t relu;          /* 1: ReLU after the (residual) add                              */
  float eps, momentum;   /* nn.BatchNorm2d eps / momentum                                 */
  int32_t dtype;         /* activations x / residual / y / g / dx / d residual: 0 fp32,
                            1 bf16 (config 3's autocast; statistics and parameters stay fp32 / fp64) */
  const void* g2;        /* backward (nullable): a second gradient of y, summed into g on load — the
                            next block's identity branch, so autograd's residual-gradient add and the
                            d residual tensor of that block never materialise (one rounding of the
                            sum to the activation type, as autograd's add)                     */
  const uint8_t* m2;     /* nullable: the next block's ReLU byte mask; g2 counts where it is 1    */
  int32_t nhwc;          /* 1: channels-last maps [N*HW][C] (C/4 a power of two, C <= 2048) — config
                            3's bf16 encoders, whose MIOpen convs then skip their NCHW<->NHWC
                            transposes.  The apply passes then take reduced sums only (ns = 1: call
                            vfd_bn_sum first); the one-launch bn1 kernels do not apply (fits = 0). */
  int32_t groups;        /* 0 / 1: one batch.  G > 1: the maps hold G consecutive batches of N images
                            each (N is the per-group count), normalised with their own statistics —
                            G separate train-mode calls of the layer in one launch (the pose net's two
                            frame pairs, models/geometry/pose.py:33-42).  partial [G][C][S][2], sums
                            [G][C+1][2] (one all-reduce for SyncBatchNorm), mean / invstd [G][C];
                            running statistics updated G times in group order, num_batches_tracked
                            += G; d gamma / d beta summed over the groups (fp32, group order). */
} vfd_bn_desc;

int vfd_bn_splits(const vfd_bn_desc* d);
int vfd_bn_fwd_stats(const vfd_bn_desc* d, const void* x, double* partial, void* stream);
/* count > 0: also writes row C = (count, 0).  invstd / dgamma / dbeta (backward, nullable): d gamma
 * = sum g'(x - mean) * invstd and d beta = sum g' from this rank's LOCAL sums (SyncBatchNorm's
 * parameter gradients are local; DDP averages them). */
int vfd_bn_sum(const vfd_bn_desc* d, const double* partial, double count, double* sums, const float* invstd,
               float* dgamma, float* dbeta, void* stream);
/* sums: the [C][S][2] partials (ns = S) or reduced [C][2] sums (ns = 1; count <= 0: the element
 * count is read from row C of the reduced sums, see vfd_bn_sum); residual / running stats
 * / num_batches_tracked (int64, += 1) nullable.  Writes y and the per-channel mean / invstd the
 * backward reads. */
/* relu_mask (optional, N*C*HW bytes): the forward also stores [y > 0] per element; a backward call
 * with d->relu == 2 then takes that mask in place of y (a quarter of the bytes). */
int vfd_bn_fwd_apply(const vfd_bn_desc* d, const void* x, const void* residual, const double* sums, int ns,
                     double count, const float* gamma, const float* beta, void* y, float* mean, float* invstd,
                     float* running_mean, float* running_var, long long* num_batches_tracked,
                     unsigned char* relu_mask, void* stream);
/* g = d y; y = the forward's output (ReLU mask; unused without ReLU), or with d->relu == 2 the
 * forward's byte mask */
int vfd_bn_bwd_stats(const vfd_bn_desc* d, const void* g, const void* y, const void* x, const float* mean,
                     double* partial, void* stream);
/* dx, d residual, d gamma, d beta nullable (not requested) */
int vfd_bn_bwd_apply(const vfd_bn_desc* d, const void* g, const void* y, const void* x, const double* sums,
                     int ns, double count, const float* gamma, const float* mean, const float* invstd, void* dx,
                     void* dresidual, float* dgamma, float* dbeta, void* stream);

/* ------------------------------------------------------------------ geometry */
/* batched 4x4 inverse of n row-major matrices (torch.inverse of the extrinsics, models/vfdepth.py:211):
 * cofactors in geometry.inverse4x4's operation order (bit-identical to it), one thread per matrix */
int vfd_inverse4x4(const float* m, float* out, int n, void* stream);

/* dtype (max pool, reflect pad, ELU + up + pad): 0 = fp32 maps, 1 = bf16 maps (config 3's autocast;
 * arithmetic in fp32, one round-to-nearest-even per output). */
/* ------------------------------------------------------------------ ResNet stem max pool */
/* MaxPool2d(3, 2, 1) of the encoders' stem, NCHW fp32: x [planes, h, w] -> y [planes, ho, wo]
 * (ho = (h-1)/2 + 1) and the winning window position (0..8) per output as one byte; ATen's tie
 * and NaN rules.  Backward: a fixed-order gather of the winners' gradients (no atomics). */
int vfd_maxpool3s2_fwd(const void* x, void* y, uint8_t* arg, long long planes, int h, int w, int dtype, void* stream);
int vfd_maxpool3s2_bwd(const void* g, const uint8_t* arg, void* dx, long long planes, int h, int w, int dtype,
                       void* stream);
/* Channels-last variants (config 3's bf16 encoders): x [n][h][w][c] -> y, arg [n][ho][wo][c], c % 4 == 0;
 * same taps, tie / NaN rules and fixed-order gather backward. */
int vfd_maxpool3s2_nhwc_fwd(const void* x, void* y, uint8_t* arg, int n, int c, int h, int w, int dtype,
                            void* stream);
int vfd_maxpool3s2_nhwc_bwd(const void* g, const uint8_t* arg, void* dx, int n, int c, int h, int w, int dtype,
                            void* stream);
/* The encoders' input normalisation (x - 0.45) / 0.225 of cat([a, b], channels) in one pass:
 * a [n_img, ca, hw], b [n_img, cb, hw] (cb = 0: a alone) -> dst [n_img, ca + cb, hw]; hw % 4 == 0. */
int vfd_normalize_cat(const float* a, const float* b, float* dst, long long n_img, int ca, int cb, int hw,
                      void* stream);

/* ------------------------------------------------------------------ reflect padding (decoders) */
/* nn.Conv2d(padding_mode='reflect', padding=1) of the decoders' 3x3 blocks (network/blocks.py):
 * x [planes, h, w] -> y [planes, h+2, w+2] (NCHW fp32), and its backward as a fixed-order gather
 * of each pixel's copies (deterministic, no atomics). */
int vfd_reflect_pad1_fwd(const void* x, void* y, long long planes, int h, int w, int dtype, void* stream);
int vfd_reflect_pad1_bwd(const void* g, void* dx, long long planes, int h, int w, int dtype, void* stream);
/* One-launch BatchNorm(+residual)(+ReLU) forward / backward for channels of at most 8192 elements
 * with local statistics (the small ResNet layers): one workgroup per channel computes the fp64
 * statistics and applies them; same arguments and results as bn_fwd_stats + bn_fwd_apply /
 * bn_bwd_stats + bn_bwd_apply (d->S unused).  vfd_bn1_fits: 1 when the shape qualifies (NCHW maps;
 * channels-last maps take the split path). */
int vfd_bn1_fits(const vfd_bn_desc* d);
int vfd_bn1_fwd(const vfd_bn_desc* d, const void* x, const void* residual, const float* gamma, const float* beta,
                void* y, float* mean, float* invstd, float* running_mean, float* running_var,
                long long* num_batches_tracked, unsigned char* relu_mask, void* stream);
int vfd_bn1_bwd(const vfd_bn_desc* d, const void* g, const void* y, const void* x, const float* gamma,
                const float* mean, const float* invstd, void* dx, void* dresidual, float* dgamma, float* dbeta,
                void* stream);

/* ------------------------------------------------------------------ disparity head (dispconv.hip) */
/* disp = sigmoid(conv3x3(xp) + b) for the decoder's full-resolution ('dispconv', 0) block
 * (fusion_depthnet.py:117-118, 139-141): xp [N, 16, H+2, W+2] already reflect-padded, w [1, 16, 3, 3],
 * out [N, 1, H, W].  Backward from g = d disp and the saved output: dxp [N, 16, H+2, W+2] (fully
 * written; NULL to skip) and partial [vfd_disp_conv_wgrad_blocks][145] = per-block sums of the 144
 * weight and the bias gradient terms (NULL to skip; the caller sums the blocks). */
int vfd_disp_conv_supported(int N, int C, int H, int W);
int vfd_disp_conv_wgrad_blocks(int N, int H, int W);
int vfd_disp_conv_fwd(const float* xp, const float* w, const float* bias, float* out, int N, int C, int H, int W,
                      void* stream);
int vfd_disp_conv_bwd(const float* g, const float* out, const float* xp, const float* w, float* dxp, float* partial,
                      int N, int C, int H, int W, void* stream);

/* ------------------------------------------------------------------ decoder convs (decconv.hip) */
/* The decoder's narrow reflect 3x3 convs (fusion_depthnet.py:97-145 upconv blocks, CI, CO in {16, 32},
 * W % 64 == 0) on fp32 MFMA (v_mfma_f32_16x16x4_f32), input already reflect-padded:
 * y [N, CO, H, W] = conv(xp [N, CI, H+2, W+2], w [CO, CI, 3, 3]) + b.  Backward from dy: dxp (all
 * padded positions; NULL to skip) and partial [vfd_dec_conv_wgrad_blocks][CO][CI][9] per-block weight
 * gradient sums (NULL to skip; the caller sums the blocks, bias gradient from the ELU kernel). */
int vfd_dec_conv_supported(int N, int CI, int CO, int H, int W);
int vfd_dec_conv_wgrad_blocks(int N, int H, int W);
int vfd_dec_conv_fwd(const float* xp, const float* w, const float* bias, float* y, int N, int CI, int CO, int H, int W,
                     void* stream);
int vfd_dec_conv_bwd(const float* dy, const float* xp, const float* w, float* dxp, float* partial, int N, int CI, int CO,
                     int H, int W, void* stream);

/* ------------------------------------------------------------------ weight relayouts (weights.hip) */
/* Once-per-step copies of reduce_dim's first-conv weight w [O, C, 3, 3] for the MFMA kernels
 * (volumetric_fusionnet.py:59-60; replace ATen permute/flip/pad chains):
 *   mode 0: K2C fragments [9][ceil16(C)/4][O][2][2] over the map's channel order; C1 > 0 means the
 *           map is z-major (z*C1 + c) and w is in the reference order c*Z + z (C = C1*Z);
 *   mode 1: K3C forward fragments [D][9][Cv/4][O][2][2] (w channel c*D + d);
 *   mode 2: K3C data-gradient copy [9 flipped taps][O/4][ceil256(Cv*D)][2][2] (n = d*Cv + c). */
int vfd_weight_fragments(int mode, const float* w, float* dst, int O, int C, int C1, int Z, int Cv, int D,
                         void* stream);
/* bf16 fragment copies (dst: bf16 elements, rounded to nearest even):
 *   mode 3: K3C forward [D][9][Cv/16][O/32][64 lanes][8]: lane l of block ob holds
 *           w[32 ob + (l & 31)][(16 q + 8 (l >> 5) + j) * D + d][tap], j = 0..7;
 *   mode 4: K2C [9][ceil32(C)/16][O/32][64 lanes][8] over the map's channel order, built from
 *           w = the fp32 mode-0 fragment copy (vfd_weight_fragments mode 0, same C / C1 / Z). */
int vfd_weight_fragments_bf16(int mode, const float* w, void* dst, int O, int C, int C1, int Z, int Cv, int D,
                              void* stream);
/* dst[o][b][a][t] = w[o][a][b][t] (w [O][A][B][taps]): the pose weight between the reference channel
 * order c*Z + z (A = C1, B = Z) and K2's map order z*C1 + c, and back for its gradient. */
int vfd_weight_swap(const float* w, float* dst, int O, int A, int B, int taps, void* stream);
/* Element (o, a, b, t) (t < T <= 9) copied from w[o*s0 + a*s1 + b*s2 + t*s3] to dst[o*d0 + a*d1 + b*d2 + t*d3]
 * (strides in floats): the swap between any NCHW / channels-last pair of layouts. */
int vfd_weight_permute(const float* w, float* dst, int O, int A, int B, int T, const long long* src_strides,
                       const long long* dst_strides, void* stream);

/* ELU(alpha 1) [+ nearest 2x upsample (up = 1)] + the one-pixel reflect pad, NCHW fp32: the
 * decoders' conv -> ELU -> upsample -> next reflect conv chain (fusion_depthnet.py:97-145,
 * blocks.py:33-38 upsample, nn.Conv2d(padding_mode='reflect')) from the conv's pre-activation
 * y [planes, h, w] straight to the next conv's padded input out [planes, (h<<up)+2, (w<<up)+2];
 * backward dy = elu'(y) * (gather of the up-block's reflect copies of g), no atomics. */
int vfd_elu_up_pad1_fwd(const void* y, void* out, long long planes, int h, int w, int up, int dtype, void* stream);
int vfd_elu_up_pad1_bwd(const void* g, const void* y, void* dy, long long planes, int h, int w, int up,
                        float* psum, int dtype, void* stream);
/* psum (optional, [planes][vfd_elu_up_pad1_bwd_blocks(h, w)]): per-block sums of dy per plane —
 * the partials of the producing conv's bias gradient (summed in fixed order by the caller) */
int vfd_elu_up_pad1_bwd_blocks(int h, int w);
/* The same chain for channels-last maps (config 3's bf16 decoders, VFD_DEC_CL): y [n_img, h, w, C]
 * -> out [n_img, (h<<up)+2, (w<<up)+2, C]; act = 0 is the plain reflect pad (ReflectPad1 on a
 * channels-last map).  C % 4 == 0, dtype 0 fp32 (16-B aligned) / 1 bf16 (8-B aligned); the
 * backward needs C / 4 to divide 256 and sums each channel's copies in the NCHW kernel's order
 * (identical d y).  y may be NULL for act 0. */
int vfd_elu_up_pad1_nhwc_fwd(const void* y, void* out, long long n_img, int h, int w, int C, int up, int act,
                             int dtype, void* stream);
int vfd_elu_up_pad1_nhwc_bwd(const void* g, const void* y, void* dy, long long n_img, int h, int w, int C, int up,
                             int act, float* part, int dtype, void* stream);
/* part (optional, [vfd_elu_up_pad1_nhwc_bwd_blocks(...)][C]): per-block channel sums of d y (bias partials) */
int vfd_elu_up_pad1_nhwc_bwd_blocks(long long n_img, int h, int w, int C);
/* backward of LeakyReLU(slope) + the one-pixel reflect pad for channels-last maps (the K3C / K2C
 * outputs): g, out [n, h+2, w+2, C] (out = the padded forward output) -> gp [n, h, w, C] =
 * (sum of g's copies) * (out > 0 ? 1 : slope); C % 4 == 0, 16-B aligned. */
int vfd_lrelu_pad1_bwd_nhwc(const float* g, const float* out, float* gp, long long n_img, int h, int w, int C,
                            float slope, void* stream);
/* the same with element types: dtype_in (g, out) / dtype_out (gp) 0 = fp32, 1 = bf16 (fp32 arithmetic,
 * one rounding of the result) */
int vfd_lrelu_pad1_bwd_nhwc_t(const void* g, const void* out, void* gp, long long n_img, int h, int w, int C,
                              float slope, int dtype_in, int dtype_out, void* stream);

/* ------------------------------------------------------------------ padded 3x3 conv (K2C) */
typedef struct vfd_conv_desc {
  int32_t B;             /* images                                                       */
  int32_t H, W;          /* rows / columns of the (already reflect-padded) input         */
  int32_t C;             /* input channels, a multiple of 4                              */
  int32_t stride;        /* 1 or 2                                                       */
  int32_t out_channels;  /* 256                                                          */
} vfd_conv_desc;

/* K2C — the pose fusion's reduce_dim[0] (volumetric_fusionnet.py:59-60, 338-343): out =
 * LeakyReLU_0.1(conv3x3_stride(x) + bias) on the reflect-padded channels-last map K2 writes,
 * x [B, H, W, C] -> out [B, Ho+2, Wo+2, 256] (Ho = (H-3)/stride + 1; reflect-padded NHWC input of
 * reduce_dim's second conv).  Wf = the weight [256, C, 3, 3] (C in x's channel order) as
 * [9 taps][Cpad/4][256][2][2] (c = 4q + 2h + s, Cpad = C rounded up to 16, zero-padded).  fp32
 * MFMA, stream-K over 16-channel chunks, fixed-order partial sums (deterministic).
 * Workspace 0 = shape unsupported. */
size_t vfd_pad_conv_fwd_workspace(const vfd_conv_desc* d);
int vfd_pad_conv_fwd(const vfd_conv_desc* d, const float* x, const float* Wf, const float* bias, float* out,
                     void* workspace, size_t ws_bytes, void* stream);
/* bf16 form (config 3's autocast): the map rounded to bf16 as it is staged, bf16 weights
 * (vfd_weight_fragments_bf16 mode 4), v_mfma_f32_32x32x16_bf16 with fp32 accumulation, bias and
 * LeakyReLU in fp32; x fp32, out bf16 (same layout as vfd_pad_conv_fwd). */
size_t vfd_pad_conv_fwd_bf16_workspace(const vfd_conv_desc* d);
int vfd_pad_conv_fwd_bf16(const vfd_conv_desc* d, const float* x, const void* Wf, const float* bias, void* out,
                          void* workspace, size_t ws_bytes, void* stream);
/* x of type dtype_x (0 fp32, 1 bf16: the map vfd_fuse_pose_fwd_t writes under config 3, C % 4 == 0). */
int vfd_pad_conv_fwd_bf16_t(const vfd_conv_desc* d, const void* x, int dtype_x, const void* Wf, const float* bias,
                            void* out, void* workspace, size_t ws_bytes, void* stream);

/* K2C data gradient (volumetric_fusionnet.py:59-60, 338-343 backward; replaces the cudnn / MIOpen
 * backward-data of the pose reduce_dim[0]): dx [B, H, W, C] (the full reflect-padded map's gradient,
 * channels-last, every position written) from g_pre [B, Ho, Wo, 256] (d pre-activation, NHWC) and Wd =
 * the weight in the MAP's channel order as vfd_weight_fragments mode 2 with Cv = C1, D = Z (the pose
 * map's z*C1 + c order; [9 flipped taps][64][np][2][2], np = C rounded up to 256).  Stride 2 by parity
 * class (4 / 2 / 2 / 1 taps), stride-K over work units, fixed-order partial sums (deterministic).
 * bf16: g_pre bf16, Wd = vfd_weight_fragments_bf16 mode 5 of that copy; dx fp32.
 * Workspace 0 = shape unsupported. */
size_t vfd_pad_conv_dgrad_workspace(const vfd_conv_desc* d);
int vfd_pad_conv_dgrad(const vfd_conv_desc* d, const float* g_pre, const float* Wd, float* dx, void* workspace,
                       size_t ws_bytes, void* stream);
size_t vfd_pad_conv_dgrad_bf16_workspace(const vfd_conv_desc* d);
int vfd_pad_conv_dgrad_bf16(const vfd_conv_desc* d, const void* g_pre, const void* Wd, float* dx, void* workspace,
                            size_t ws_bytes, void* stream);
/* dtype_dx 0: fp32 dx (as vfd_pad_conv_dgrad_bf16), 1: bf16 dx — the fp32 sums rounded once to
 * nearest even, as a bf16 convolution's input gradient under autocast (config 3's pose map) */
int vfd_pad_conv_dgrad_bf16_t(const vfd_conv_desc* d, const void* g_pre, const void* Wd, void* dx, int dtype_dx,
                              void* workspace, size_t ws_bytes, void* stream);

/* K3C data gradient (volumetric_fusionnet.py:59-60, 265 backward): d of reduce_dim's first conv
 * w.r.t. its reflect-padded input, dx [B*N, h+2, w+2, D*Cv] (channel d*Cv + c: the layout
 * vfd_voxel_project_bwd_planned reads) from g_pre [B*N, h, w, O = 256] (d pre-activation, NHWC)
 * and Wd = the weight [O, Cv*D, 3, 3] as [9 flipped taps][O/4][np][2][2] (np = D*Cv rounded up
 * to 256, zero-padded).  fp32 MFMA, stream-K with a fixed-order partial sum (deterministic).
 * d->pad_out == 2: the folded form — only the interior of dx is written, each border-adjacent pixel
 * holding the sum of its reflect copies (the plan for vfd_voxel_project_bwd_planned must be built
 * with the same pad_out): tiles of 256 interior pixels x 128 channels, any h, w >= 2 whose staged
 * rows fit LDS (w <= 128; config 5's 80 x 120 included).
 * Workspace 0 = shape unsupported (Cv != 64, D > 64, or the staged rows of a tile exceed LDS). */
size_t vfd_proj_conv_dgrad_workspace(const vfd_voxel_desc* d);
int vfd_proj_conv_dgrad(const vfd_voxel_desc* d, const float* g_pre, const float* Wd, float* dx, void* workspace,
                        size_t ws_bytes, void* stream);

/* bf16 form of the folded K3C data gradient (config 3; d->pad_out must be 2): g_pre bf16
 * [B*N, h, w, O] NHWC, Wd = vfd_weight_fragments_bf16 mode 5 of the mode-2 copy, v_mfma_f32_32x32x16_bf16
 * with fp32 accumulation, dx fp32 (the interior of [B*N, h+2, w+2, D*Cv], as vfd_proj_conv_dgrad).
 * Workspace 0 = shape unsupported. */
size_t vfd_proj_conv_dgrad_bf16_workspace(const vfd_voxel_desc* d);
int vfd_proj_conv_dgrad_bf16(const vfd_voxel_desc* d, const void* g_pre, const void* Wd, float* dx, void* workspace,
                             size_t ws_bytes, void* stream);

/* bf16 weight / bias gradients (config 3; MIOpen's bf16 weight gradient before): K3C from g_pre bf16
 * [B*N, h, w, O] and the bf16 frustum side output x [B*N, h+2, w+2, D*Cv] into dw [O, Cv*D, 3, 3] fp32
 * in the reference channel order c*D + d; K2C from g_pre bf16 [B, Ho, Wo, 256] and the fp32 padded BEV
 * map x [B, H, W, C] (rounded to bf16 as staged) into dw_map [256, C, 3, 3] fp32 in the MAP's channel
 * order (the caller swaps it to the reference's c*Z + z).  db [O] fp32 (nullable, as dw).
 * v_mfma_f32_32x32x16_bf16 on transposed LDS reads, stream-K, fixed-order sums (deterministic). */
size_t vfd_proj_conv_wgrad_bf16_workspace(const vfd_voxel_desc* d);
int vfd_proj_conv_wgrad_bf16(const vfd_voxel_desc* d, const void* g_pre, const void* x, float* dw, float* db,
                             void* workspace, size_t ws_bytes, void* stream);
size_t vfd_pad_conv_wgrad_bf16_workspace(const vfd_conv_desc* d);
int vfd_pad_conv_wgrad_bf16(const vfd_conv_desc* d, const void* g_pre, const float* x, float* dw_map, float* db,
                            void* workspace, size_t ws_bytes, void* stream);
/* x of type dtype_x (0 fp32, 1 bf16 map). */
int vfd_pad_conv_wgrad_bf16_t(const vfd_conv_desc* d, const void* g_pre, const void* x, int dtype_x, float* dw_map,
                              float* db, void* workspace, size_t ws_bytes, void* stream);

/* K3C weight / bias gradient (volumetric_fusionnet.py:59-60, 265 backward; replaces the
 * reference's cudnn weight-gradient of reduce_dim[0]): dw [O = 256, Cv*D, 3, 3] in the reference
 * channel order c*D + d, db [O], from g_pre [B*N, h, w, O] (NHWC) and the frustum features x
 * [B*N, h+2, w+2, D*Cv] that vfd_proj_conv_fwd wrote as x_out.  fp32 MFMA, stream-K with a
 * fixed-order partial sum (deterministic).  dw or db may be null (not computed).
 * Workspace 0 = shape unsupported (Cv != 64 or D > 64). */
size_t vfd_proj_conv_wgrad_workspace(const vfd_voxel_desc* d);
int vfd_proj_conv_wgrad(const vfd_voxel_desc* d, const float* g_pre, const float* x, float* dw, float* db,
                        void* workspace, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------ view synthesis (K4) */
typedef struct vfd_view_desc {
  int32_t B, N, H, W;
  int32_t n_warp;        /* warps per target camera                                      */
  int32_t n_temporal;    /* T = len(frame_ids) - 1 temporal warps (warps 0..T-1)         */
  int32_t n_overlap;     /* overlap slots: len(frame_ids) when spatial terms are on, else 0 */
  int32_t intensity_align;
  int32_t cam_begin;     /* target cameras cam_begin .. cam_begin+cam_count-1 are rendered */
  int32_t cam_count;     /* (per-target arrays are [B, cam_count, ...])                  */
  const float* color[4]; /* per frame slot (frame_ids order) [B, N, 3, H, W]             */
  const int32_t* warp_tab; /* [N, n_warp, 3] device: frame slot, source camera, overlap slot (-1: temporal) */
} vfd_view_desc;

/* Projection.forward + get_virtual_image + get_norm_image_single + overlap accumulation
 * (models/geometry/geometry_util.py:52-82, view_rendering.py:30-82, 118-198) for every target
 * camera and warp in three fused passes.  With Nt = cam_count target cameras:
 * depth [B,Nt,H,W], invK [B,Nt,4,4] (scale 0), M [B,Nt,n_warp,3,4] = (K_src @ T)[:3],
 * mask [B,N,H,W] (all cameras).
 * Outputs: color [B,Nt,T,3,H,W], cmask [B,Nt,T,H,W], ovl [B,Nt,F,3,H,W], omask [B,Nt,F,H,W];
 * coef [B,Nt,n_warp,4] (w_mean, w_std, s_mean, s_std; w_std < 0: warp left unnormalised). */
size_t vfd_view_workspace_bytes(const vfd_view_desc* d);
int vfd_view_fwd(const vfd_view_desc* d, const float* depth, const float* invK, const float* M,
                 const float* mask, float* color, float* cmask, float* ovl, float* omask,
                 float* coef, void* workspace, size_t ws_bytes, void* stream);
/* g_color [B,Nt,T,3,H,W], g_ovl [B,Nt,F,3,H,W] (nullable) -> d_depth [B,Nt,H,W], d_M [B,Nt,n_warp,3,4]. */
int vfd_view_bwd(const vfd_view_desc* d, const float* depth, const float* invK, const float* M,
                 const float* mask, const float* coef, const float* g_color, const float* g_ovl,
                 float* d_depth, float* d_M, void* workspace, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------ depth synthesis (aug_depth) */
typedef struct vfd_depthsyn_desc {
  int32_t B, N, H, W;
  int32_t S;             /* source slots per target camera (rel_cam_list[c] + [c])          */
  float min_depth, max_depth;   /* training.min_depth / max_depth                          */
  const int32_t* src_tab;       /* [N, S] device: source camera of each slot (-1: absent)  */
} vfd_depthsyn_desc;

/* get_virtual_depth for every (target camera, source slot) (view_rendering.py:84-116, 201-241):
 * aug_depth [B,N,H,W] (depth at the augmented view of each camera), depth [B,N,H,W] (each
 * camera's depth), mask [B,N,H,W], invK [B,N,4,4] (scale 0), M [B,N,S,3,4] = (K_src @ T^-1)[:3],
 * zrow [B,N,S,4] = T[2, :] with T = E_aug[c]^-1 E[src]  ->  tform_depth, tform_mask [B,N,S,H,W]. */
int vfd_depth_syn_fwd(const vfd_depthsyn_desc* d, const float* aug_depth, const float* depth, const float* mask,
                      const float* invK, const float* M, const float* zrow, float* tform_depth, float* tform_mask,
                      void* stream);
/* g [B,N,S,H,W] (d tform_depth) -> d_aug [B,N,H,W] (written), d_depth [B,N,H,W] (zeroed here, atomics). */
int vfd_depth_syn_bwd(const vfd_depthsyn_desc* d, const float* aug_depth, const float* depth, const float* mask,
                      const float* invK, const float* M, const float* zrow, const float* g, float* d_aug,
                      float* d_depth, void* stream);
/* The same backward with d_depth summed in exact 128-bit fixed point (2^-100 resolution, |sum| < 2^26;
 * integer adds, so the result does not depend on the order the scattered contributions land in):
 * the deterministic mode's form (torch.backends.cudnn.deterministic / VFD_DETERMINISTIC=1).
 * workspace >= vfd_depth_syn_bwd_ordered_workspace(d) bytes (16 per source pixel). */
size_t vfd_depth_syn_bwd_ordered_workspace(const vfd_depthsyn_desc* d);
int vfd_depth_syn_bwd_ordered(const vfd_depthsyn_desc* d, const float* aug_depth, const float* depth,
                              const float* mask, const float* invK, const float* M, const float* zrow,
                              const float* g, float* d_aug, float* d_depth, void* workspace, size_t ws_bytes,
                              void* stream);

/* ------------------------------------------------------------------ photometric losses (K5) */
typedef struct vfd_photo_desc {
  int32_t B, N, H, W;
  int32_t T;             /* temporal frames (frame_ids[1:])                              */
  int32_t F;             /* overlap slots (0 = SingleCamLoss)                            */
  int32_t cam_begin;     /* target cameras cam_begin .. cam_begin+cam_count-1            */
  int32_t cam_count;
  uint64_t seed;         /* identity-noise RNG seed, used when `noise` is NULL            */
  const int64_t* step;   /* optional device step counter mixed into the seed (graph replay) */
  float noise_scale;     /* 1e-5 (single_cam_loss.py:8)                                  */
  const float* ident[4]; /* identity sources per temporal frame [B, N, 3, H, W]          */
} vfd_photo_desc;

/* compute_photometric_loss / compute_ssim_loss / auto-mask / masked means for every camera
 * (models/losses/loss_util.py:6-78, single_cam_loss.py:17-55, multi_cam_loss.py:16-59).
 * With Nt = cam_count: target [B,N,3,H,W] and ref_mask [B,N,H,W] (all cameras);
 * color [B,Nt,T,3,H,W]; ovl [B,Nt,F,3,H,W]; omask [B,Nt,F,H,W]; noise [Nt,B,T,H,W] or NULL.
 * Outputs: reproj [B,Nt,H,W] (automask * min reprojection), automask [B,Nt,H,W],
 * spatio_mask [B,Nt,H,W], sel [B,Nt,H,W] uint8 (argmin bits, saved for backward),
 * sums [Nt, 6] double (S_reproj, M_reproj, S_spatio, M_spatio, S_st, M_st),
 * losses [Nt, 3] float (reproj, spatio, spatio-temporal masked means). */
size_t vfd_photo_workspace_bytes(const vfd_photo_desc* d);
int vfd_photo_fwd(const vfd_photo_desc* d, const float* target, const float* color,
                  const float* ovl, const float* ref_mask, const float* omask, const float* noise,
                  float* reproj, float* automask, float* spatio_mask, uint8_t* sel, double* sums,
                  float* losses, void* workspace, size_t ws_bytes, void* stream);
/* gcoef [Nt, 3] = upstream grad / (mask sum + 1e-8) per term -> d_color, d_ovl (overwritten). */
int vfd_photo_bwd(const vfd_photo_desc* d, const float* target, const float* color,
                  const float* ovl, const float* ref_mask, const float* omask, const uint8_t* sel,
                  const float* gcoef, float* d_color, float* d_ovl, void* stream);

/* Edge-aware smoothness of disp / mean(disp) (loss_util.py:28-40, single_cam_loss.py:57-65).
 * disp [B,N,H,W], color [B,N,3,H,W] -> sums [B*N, 3] double (sum disp, Sx, Sy), loss [N]. */
size_t vfd_smooth_workspace_bytes(int B, int N, int H, int W);
int vfd_smooth_fwd(int B, int N, int H, int W, const float* disp, const float* color,
                   double* sums, float* loss, void* workspace, size_t ws_bytes, void* stream);
/* g [N] upstream grads -> d_disp [B,N,H,W] (overwritten). */
int vfd_smooth_bwd(int B, int N, int H, int W, const float* disp, const float* color,
                   const double* sums, const float* g, float* d_disp, void* stream);

/* ------------------------------------------------------------------ feature aggregation */
/* LReLU_0.1(base + sum_k up_align_corners(level_k) + bias) at the fusion level
 * (network/fusion_depthnet.py:53-63: 1x1 conv of the concatenated, upsampled pyramid, with the
 * conv applied per level by the caller).  base/out [BN, C, h, w]; levels[k] [BN, C, level_hw[2k],
 * level_hw[2k+1]] (host array of device pointers), n_levels <= 3; bias [C]. */
int vfd_aggregate_fwd(int BN, int C, int h, int w, const float* base, int n_levels,
                      const float* const* levels, const int* level_hw, const float* bias, float* out,
                      void* stream);
/* the same with channels-last inputs read in place: base [BN, h, w, C], levels[k] [BN, hs, ws, C] of
 * dtype 0 fp32 / 1 bf16 (config 3's bf16 1x1-conv products), out NCHW fp32 [BN, C, h, w]; per
 * element the arithmetic of vfd_aggregate_fwd on the fp32 values (bit-identical). */
/* x NCHW fp32 [n][C][hw] -> y channels-last [n][hw][C] of dtype_out (0 fp32, 1 bf16, rounded to
 * nearest even): AggregateUp's input gradients in the layout / dtype of its channels-last inputs */
int vfd_nchw_to_nhwc(const float* x, void* y, long long n, int C, int hw, int dtype_out, void* stream);
int vfd_aggregate_fwd_cl(int BN, int C, int h, int w, const void* base, int n_levels, const void* const* levels,
                         const int* level_hw, const float* bias, float* out, int dtype, void* stream);
/* backward of vfd_aggregate_fwd in one launch (one workgroup per plane, LDS-resident):
 * d = g * LReLU'(out) [BN, C, h, w] (the base's gradient), psum [BN * C] = its plane sums (the
 * caller sums them over n for the bias gradient), dlevels[k] [BN, C, level_hw[2k], level_hw[2k+1]]
 * = the upsample adjoint of d (the fixed-order separable gather of vfd_upsample_ac_bwd).
 * Needs (h * w + h * max_k level_w + 5 * (h + w)) * 4 <= 64 KiB (else VFD_EINVAL). */
int vfd_aggregate_bwd(int BN, int C, int h, int w, const float* g, const float* out, float* d, int n_levels,
                      float* const* dlevels, const int* level_hw, float* psum, void* stream);
/* backward of the align_corners bilinear upsample (the aggregation's levels): g [planes, h, w] ->
 * dsrc [planes, hs, ws] as a separable fixed-order gather (deterministic, no atomics);
 * tmp: [planes, h, ws] scratch */
int vfd_upsample_ac_bwd(const float* g, float* dsrc, float* tmp, long long planes, int h, int w, int hs, int ws,
                        void* stream);

/* ------------------------------------------------------------------ measurement hooks */
/* Record HIP events around every launch of kernel `kernel_id` (see vfd_kernel_name; -1 = all,
 * -2 = off) on the launching stream.  vfd_prof_read: launches and summed ms of everything
 * recorded; vfd_prof_read_kernels: the same per kernel id into arrays of `count` entries.
 * Both reset the record. */
#define VFD_PROF_ALL (-1)
#define VFD_KERNEL_COUNT 33
const char* vfd_kernel_name(int kernel_id);
int vfd_prof_enable(int kernel_id);
int vfd_prof_read(int* launches, double* total_ms);
int vfd_prof_read_kernels(int count, int* launches, double* total_ms);

#ifdef __cplusplus
}
#endif
#endif /* VFD_CAPI_H */
