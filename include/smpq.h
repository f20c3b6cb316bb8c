/*
 * smpq.h — C-ABI of libsmpq.so, the MI355X-native (gfx950) semilayer mixed-precision
 * quantized convolution library.
 *
 * Plain pointers and sizes only (no torch types). Every device pointer is owned by the
 * caller (PyTorch's caching allocator on the Python side); the library never allocates
 * device memory and keeps no pointer past a call. Every kernel is enqueued on the HIP
 * stream passed in (Python passes torch.cuda.current_stream().cuda_stream), nothing blocks
 * the host except the *_host entry points. Return value: 0 on success, a negative SMPQ_E_*
 * code otherwise; smpq_last_error() holds a thread-local message.
 *
 * Reference interfaces replaced (kenm-28/Semilayer-Wise-Mixed-Precision-Quantization):
 *   smpq_quantize_channels[_host]  functions.py:25-43 quantize_wgt, applied per output channel
 *                                  as functions.py:9-23 channel_wise_quantizationperchan does
 *                                  (called from resnet50_main.py:189-197, functions.py:504-512)
 *   smpq_pack_weights              (new) fake-quantized fp32 weight -> int8 codes + per-channel
 *                                  step/offset; feeds the conv below (the reference keeps the
 *                                  fake-quantized fp32 weight in nn.Conv2d, resnet.py:22-30)
 *   smpq_conv2d_fwd                nn.Conv2d forward on the fake-quantized weight
 *                                  (resnet.py:22-30 via resnet.py:57,60,99,103,107) fused with
 *                                  the eval BatchNorm / ReLU / residual add that follow it in
 *                                  BasicBlock.forward (resnet.py:55-68) / Bottleneck.forward
 *                                  (resnet.py:97-116)
 *   smpq_act_absmax                (new) per-image activation range for the activation quantizer
 *   smpq_act_quantize              (new) activation quantizer (the reference keeps fp32 activations;
 *                                  int16/int24 codes reproduce them within the stated tolerance)
 *   smpq_softmax_xent              per-batch body of functions.py:84-129 evaluate_acc_loss_softmax
 *                                  (output.max(1), CrossEntropyLoss, Softmax(dim=1), :113-121)
 *   smpq_kl_rows                   functions.py:131-149 KLdiv (per-image sum_c n*log(n/o), :140-146)
 *   smpq_avgpool_fc                avgpool + flatten + fc of ResNet._forward_impl (resnet.py:216-218),
 *                                  batch-invariant (sharded logits == single-GPU logits, bitwise)
 */
#ifndef SMPQ_H_
#define SMPQ_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SMPQ_ABI_VERSION 7

/* status codes */
#define SMPQ_OK 0
#define SMPQ_E_INVALID (-1)  /* bad argument / unsupported configuration */
#define SMPQ_E_SHAPE (-2)    /* shape the kernels do not support */
#define SMPQ_E_BITS (-3)     /* bit-width outside {1..8} */
#define SMPQ_E_RANGE (-4)    /* a channel's codes span more than 256 levels */
#define SMPQ_E_CONSTANT (-5) /* constant channel: the reference raises ZeroDivisionError */
#define SMPQ_E_HIP (-6)      /* a HIP runtime call failed */
#define SMPQ_E_INEXACT (-7)  /* weights are not on the recorded quantization grid */

typedef void* smpq_stream_t; /* hipStream_t */

int smpq_abi_version(void);
const char* smpq_last_error(void);
/* SHA-256 (hex) of the sources, headers and compiler flags this library was built from;
 * __graft_entry__.build() rebuilds whenever the tree's hash differs from it. */
const char* smpq_build_stamp(void);

/* Rounding semantics of functions.py:41 `t / scale` (scale a Python float), which depend on
 * where the reference's tensor lives:
 *   SMPQ_QSEM_CPU     torch on the CPU: IEEE fp32 division t / fp32(scale)
 *   SMPQ_QSEM_DEVICE  torch on the GPU: t * fp32(1.0 / scale) (reciprocal of the double scale,
 *                     rounded once; tests/golden/quant_kat_device.npz, produced by torch on an
 *                     MI355X, pins it) */
#define SMPQ_QSEM_CPU 0
#define SMPQ_QSEM_DEVICE 1

/* Fake-quantize channels of w in place, bit-exactly as functions.py:25-43 executes under
 * `semantics` (SMPQ_QSEM_*).
 *   w          device fp32 [cout][k_elems] (one output channel per row)
 *   bits       device int8 [cout]; 0 leaves the channel untouched
 *   scale_out  device fp32 [cout]; receives fp32(scale) of the quantization applied
 *   status     device int32 [1], caller-zeroed; set to (first constant channel)+1 */
int smpq_quantize_channels_ex(float* w, int cout, int k_elems, const int8_t* bits,
                              float* scale_out, int32_t* status, int semantics, smpq_stream_t stream);

/* smpq_quantize_channels_ex with SMPQ_QSEM_CPU (ABI v1 entry point, kept). */
int smpq_quantize_channels(float* w, int cout, int k_elems, const int8_t* bits,
                           float* scale_out, int32_t* status, smpq_stream_t stream);

/* Host-memory twin of smpq_quantize_channels (same arithmetic, native C++), used when the
 * weight lives in host memory (the reference quantizes CPU tensors of fresh models, e.g.
 * functions.py:504-512 right after resnet.resnet50(...) at :528). Returns SMPQ_E_CONSTANT on
 * a constant channel (channels before it are already quantized, as in the reference loop). */
int smpq_quantize_channels_host_ex(float* w, int cout, int k_elems, const int8_t* bits,
                                   float* scale_out, int semantics);

/* smpq_quantize_channels_host_ex with SMPQ_QSEM_CPU (ABI v1 entry point, kept). */
int smpq_quantize_channels_host(float* w, int cout, int k_elems, const int8_t* bits,
                                float* scale_out);

/* Pack fake-quantized weights into the conv kernel's layout.
 *   w       device fp32 [cout][cin][kh][kw] (fake-quantized, values fl32(m * step))
 *   step    device fp32 [cout] quantization step (scale_out of the quantizer)
 *   codes   device int8 [cout][kh][kw][cin]   m - offset, in [-128, 127]
 *   offset  device int32 [cout]
 *   status  device int32 [2], caller-zeroed: [0] += channels not on the grid,
 *           [1] += channels whose codes span > 256 levels */
int smpq_pack_weights(const float* w, int cout, int cin, int kh, int kw, const float* step,
                      int8_t* codes, int32_t* offset, int32_t* status, smpq_stream_t stream);

/* General weight packer for smpq_conv2d_fwd_ex: `wlimbs` int8 planes codes[wlimbs][cout][K].
 *   step     device fp32 [cout] recorded quantization step, 0 = never quantized (may be NULL
 *            when wlimbs == 2: every channel then uses 16-bit fixed point)
 *   wlimbs   1: exact int8 codes (m - offset) of quantized channels (status[0]/[1] report
 *            channels that cannot be coded); 2 / 3: exact codes of quantized channels that fit
 *            16 / 24 bits, per-channel fixed point (max|w| / 32512 or / 8323072) for the others
 *            (status[2] counts them)
 *   cin      a multiple of 64 (K = kh*kw*cin, ordered [kh][kw][cin]); the <= 4-channel stem is
 *            packed by smpq_pack_weights_s2d_ex
 *   offset   device int32 [cout] (wlimbs == 1), wscale device fp32 [cout]: the per-channel weight
 *            step the codes are in (= step for exact channels)
 *   status   device int32 [3], caller-zeroed */
int smpq_pack_weights_ex(const float* w, int cout, int cin, int kh, int kw, const float* step,
                         int wlimbs, int8_t* codes, int32_t* offset, float* wscale, int32_t* status,
                         smpq_stream_t stream);

/* Per-image absolute maximum, accumulated with atomicMax into absmax[n] (caller zeroes). */
int smpq_act_absmax(const float* x, int n, int64_t per_image, float* absmax,
                    smpq_stream_t stream);

/* Activation quantizer: q = clamp(rne(x * QMAX_L / absmax[img]), +-QMAX_L) with
 * QMAX_1 = 127, QMAX_2 = 32512, QMAX_3 = 8323072, written as `limbs` balanced base-256 int8
 * digit planes (q = sum_l 256^l * plane_l), each plane laid out like x.
 *   x        device fp32, n images of per_image elements (per_image % 8 == 0)
 *   absmax   device fp32 [n] (from smpq_act_absmax or a conv's y_absmax)
 *   out      device int8 [limbs][n * per_image] */
int smpq_act_quantize(const float* x, int n, int64_t per_image, const float* absmax, int limbs,
                      int8_t* out, smpq_stream_t stream);

/* MaxPool2d(3, stride 2, pad 1) (resnet.py:147) on NHWC fp32 [n][h][w][c] (c % 4 == 0), fused
 * with the activation quantizer of its output: `limbs` int8 planes [n][ho][wo][c] with the
 * per-image range absmax (the pool input's max; equal to the output's for ReLU outputs).
 * out_f32: optional fp32 NHWC pooled output (NULL to skip). */
int smpq_maxpool_quantize(const float* x, int n, int h, int w, int c, const float* absmax, int limbs,
                          int8_t* out, float* out_f32, smpq_stream_t stream);

/* Quantized conv forward (implicit GEMM on int8 MFMA), NHWC.
 *   xq         device int8 [limbs][n][h][w][cin] digit planes from smpq_act_quantize; cin % 64 == 0
 *   x_absmax   device fp32 [n]: the per-image range xq was quantized with
 *   codes/offset/cout/kh/kw: from smpq_pack_weights (offset may be NULL when all zero)
 *   col_scale  device fp32 [cout]: y = conv_real * col_scale[c] + col_shift[c]
 *              (col_scale = step * bn_gamma / sqrt(var+eps), col_shift = bn_beta - mean * ...)
 *   residual   device fp32 NHWC [n][ho][wo][cout] added after the affine, or NULL
 *   relu       0/1, applied last
 *   limbs      activation code width in int8 limbs: 1 (int8), 2 (int16), 3 (int24)
 *   y          device fp32 NHWC [n][ho][wo][cout]
 *   y_absmax   device fp32 [n] (caller-zeroed), receives max|y| per image, or NULL
 *   tile_cfg   block tile configuration (smpq_conv2d_tile_config), or -1 for the built-in choice
 *   cout % 16 == 0, and every activation / output plane below 2 GiB (32-bit buffer offsets:
 *   SMPQ_E_SHAPE otherwise; the Python layer splits such batches). ABI v4: the register-staged
 *   kernel family of v1-v3 (and with it cin == 4) is gone; tile configurations are numbered from 0
 *   in the LDS-DMA family. */
int smpq_conv2d_fwd(const int8_t* xq, const float* x_absmax, int n, int h, int w, int cin,
                    const int8_t* codes, const int32_t* offset, int cout, int kh, int kw,
                    int stride, int pad, const float* col_scale, const float* col_shift,
                    const float* residual, int relu, int limbs, float* y, float* y_absmax,
                    int tile_cfg, smpq_stream_t stream);

/* smpq_conv2d_fwd with weight limbs (1, 2, or 3 with limbs == 3): codes [wlimbs][cout][K] from
 * smpq_pack_weights_ex. col_scale must include the per-channel weight step (wscale) of the
 * packer. */
int smpq_conv2d_fwd_ex(const int8_t* xq, const float* x_absmax, int n, int h, int w, int cin,
                       const int8_t* codes, int wlimbs, const int32_t* offset, int cout, int kh,
                       int kw, int stride, int pad, const float* col_scale, const float* col_shift,
                       const float* residual, int relu, int limbs, float* y, float* y_absmax,
                       int tile_cfg, smpq_stream_t stream);

/* smpq_conv2d_fwd_ex that can also (or only) emit the NEXT conv's activation limb planes:
 *   y          fp32 NHWC output, or NULL when only yq is wanted
 *   yq         int8 [limbs][n*ho*wo][cout] planes of q = clamp(rne(y * QMAX / yq_range)), or NULL
 *   yq_range   static per-layer range (> 0) of the output quantizer (calibrated by the caller)
 *   overflow   device int32 [1]: set to 1 when some |y| > yq_range (values are then clamped; the
 *              caller re-runs with dynamic ranges)
 *   residual_q int8 [limbs][n*ho*wo][cout] limb planes of the residual (e.g. the block input as
 *              written by the previous conv's yq), dequantized as residual_range/QMAX * q; NULL
 *              when `residual` (fp32) or no residual is used */
int smpq_conv2d_fwd_q(const int8_t* xq, const float* x_absmax, int n, int h, int w, int cin,
                      const int8_t* codes, int wlimbs, const int32_t* offset, int cout, int kh,
                      int kw, int stride, int pad, const float* col_scale, const float* col_shift,
                      const float* residual, int relu, int limbs, float* y, float* y_absmax,
                      int8_t* yq, float yq_range, int32_t* overflow, const int8_t* residual_q,
                      float residual_range, int tile_cfg, smpq_stream_t stream);

/* smpq_conv2d_fwd_q with a second copy of the same codes in the K-major layout
 * codes_kmajor [wlimbs][K/64][cout][64] (smpq_weights_kmajor; round 3): the LDS-DMA tile
 * configurations then stage every weight piece from whole cache lines (the 64-B K slices of 16
 * consecutive output channels are one contiguous KiB) instead of 16 half lines — 6-21 % faster
 * on the MFMA-heavy convs. Results are bitwise those of smpq_conv2d_fwd_q. codes (row-major) is
 * still required (the v3 signature is kept); codes_kmajor may be NULL. */
int smpq_conv2d_fwd_q_km(const int8_t* xq, const float* x_absmax, int n, int h, int w, int cin,
                         const int8_t* codes, const int8_t* codes_kmajor, int wlimbs, const int32_t* offset,
                         int cout, int kh, int kw, int stride, int pad, const float* col_scale,
                         const float* col_shift, const float* residual, int relu, int limbs, float* y,
                         float* y_absmax, int8_t* yq, float yq_range, int32_t* overflow,
                         const int8_t* residual_q, float residual_range, int tile_cfg, smpq_stream_t stream);

/* ABI 7: a Bottleneck's conv3 (+ limb-plane identity, ReLU) chained with the NEXT block's conv1
 * (ReLU) in one launch (resnet.py:111-113, then :99-101 of the next block): the second conv reads
 * the first one's output tile from LDS instead of HBM. Both outputs and the overflow flag are
 * bitwise those of two smpq_conv2d_fwd_q calls. 3 activation limbs, exact weight codes (no offsets):
 *   xq, x_absmax, n, h, w, cin          conv3's input, as smpq_conv2d_fwd_q (1x1, stride 1, pad 0)
 *   codes1 [cout1][cin], col_scale1, col_shift1 [cout1]        conv3 (+ its folded BN)
 *   residual_q [3][n*h*w][cout1], residual_range               the identity's limb planes
 *   yq1 [3][n*h*w][cout1], yq1_range    conv3's output limb planes (the next block's identity)
 *   y1_absmax [n]                       per-image range conv1 reads them with (what a separate
 *                                       conv1 launch gets as x_absmax)
 *   codes2 [cout2][cout1], col_scale2, col_shift2 [cout2]      the next block's conv1
 *   yq2 [3][n*h*w][cout2], yq2_range    conv1's output limb planes
 *   overflow                            int32 [1]: set when either output exceeded its range
 * Built for (cin, cout1, cout2) = (64, 256, 64) and (64, 256, 128), the ResNet-50 layer1 blocks and
 * layer 1's last conv3 with layer 2's first conv1 (smpq_conv2d_pair_supported); other calls return
 * SMPQ_E_INVALID. */
int smpq_conv2d_pair_supported(int cin, int cout1, int cout2, int limbs);
int smpq_conv2d_pair_fwd(const int8_t* xq, const float* x_absmax, int n, int h, int w, int cin,
                         const int8_t* codes1, int cout1, const float* col_scale1, const float* col_shift1,
                         const int8_t* residual_q, float residual_range, int8_t* yq1, float yq1_range,
                         const float* y1_absmax, const int8_t* codes2, int cout2, const float* col_scale2,
                         const float* col_shift2, int8_t* yq2, float yq2_range, int32_t* overflow,
                         smpq_stream_t stream);

/* ABI 7: the general form of the Bottleneck tail chain. conv3 (exact codes; offset1 = its weight
 * offsets or NULL) with its identity from ONE of
 *   residual_q / residual_range        the identity's limb planes, as smpq_conv2d_pair_fwd, or
 *   ds_xq [3][n*ds_h*ds_w][ds_cin], ds_x_absmax [n], ds_codes [3][cout1][ds_cin] (ds_wlimbs = 3:
 *   24-bit fixed point from smpq_pack_weights_ex), ds_col_scale / ds_col_shift [cout1], ds_range
 *                                      the block's 1x1 downsample (stride ds_stride) whose output
 *                                      pixels are conv3's, computed in the same tiles: its clamped
 *                                      output codes (what a
 *                                      smpq_conv2d_fwd_q launch with emit range ds_range writes) are
 *                                      conv3's residual and are never written; overflow covers them,
 * and optionally (codes2 != NULL) the next block's conv1 on conv3's output as smpq_conv2d_pair_fwd
 * (no offsets). Every output and the overflow flag are bitwise those of the separate launches.
 * Built: conv3 64 -> 256 with the next conv1 256 -> 64 or 256 -> 128 (smpq_conv2d_chain_supported), and conv3
 * with a fused downsample and no second conv for the first blocks of R50's layers 1-3 (64 -> 256 /
 * ds 64 / stride 1, 128 -> 512 / ds 256 / 2, 256 -> 1024 / ds 512 / 2: smpq_conv2d_chain_ds_supported);
 * other calls return SMPQ_E_INVALID. */
int smpq_conv2d_chain_supported(int cin, int cout1, int cout2, int limbs);
int smpq_conv2d_chain_ds_supported(int cin, int cout1, int ds_cin, int ds_stride, int limbs);
int smpq_conv2d_chain_fwd(const int8_t* xq, const float* x_absmax, int n, int h, int w, int cin,
                          const int8_t* codes1, const int32_t* offset1, int cout1, const float* col_scale1,
                          const float* col_shift1, const int8_t* residual_q, float residual_range,
                          const int8_t* ds_xq, const float* ds_x_absmax, int ds_h, int ds_w, int ds_cin,
                          int ds_stride, const int8_t* ds_codes, int ds_wlimbs,
                          const float* ds_col_scale, const float* ds_col_shift, float ds_range, int8_t* yq1,
                          float yq1_range, const float* y1_absmax, const int8_t* codes2, int cout2,
                          const float* col_scale2, const float* col_shift2, int8_t* yq2, float yq2_range,
                          int32_t* overflow, smpq_stream_t stream);

/* codes [wlimbs][cout][K] (K % 64 == 0, 16-B aligned) -> out [wlimbs][K/64][cout][64], the K-major
 * copy smpq_conv2d_fwd_q_km reads. */
int smpq_weights_kmajor(const int8_t* codes, int wlimbs, int cout, int K, int8_t* out, smpq_stream_t stream);

/* 3x3 / stride 2 / pad 1 max pool (resnet.py:147) directly on int8 limb planes
 * x [limbs][n][h][w][c] -> out [limbs][n][ho][wo][c], c % 16 == 0 (static-range mode: the codes of
 * one activation share one step, so the max of the codes is the code of the max — exact). */
int smpq_maxpool_limbs(const int8_t* x, int n, int h, int w, int c, int limbs, int8_t* out, smpq_stream_t stream);

/* ---- space-to-depth stem (the 7x7 / stride 2 / pad 3 conv1 of resnet.py:143) -------------------
 * The stem runs as a 4x4 / stride 1 conv over 16-channel "space-to-depth" pixels (each a 2x2
 * block of the image with up to 4 channels), so every 64-byte K step of the int8 GEMM is one
 * tap row of whole 16-byte pixels (tests/test_gpu.py checks it against an exact emulation of the
 * 7x7/2/3 conv on the quantized image).
 *
 * smpq_image_quantize_s2d: x fp32 NCHW [n][c <= 4][h][w] (h, w >= 2) ->
 *   out int8 [limbs][n][ceil(h/2)][ceil(w/2)][16], channel (dy*2 + dx)*4 + ci = x[ci][2i + dy][2j + dx]
 *   quantized with the per-image absmax as smpq_act_quantize does (zero for ci >= c and past an
 *   odd h or w: the conv's own zero padding).
 * smpq_pack_weights_s2d_ex: w fp32 [cout][cin <= 4][7][7] -> codes int8 [wlimbs][cout][256] (K order
 *   [ty][tx][dy][dx][ci], original tap (2 ty + dy - 1, 2 tx + dx - 1), zero outside 7x7) with scale
 *   wscale [cout]: channels with a recorded quantization step (step[c] > 0; step may be NULL) as
 *   exact codes, the others in per-channel fixed point (wlimbs 2 / 3 = 16 / 24 bits) — the rules of
 *   smpq_pack_weights_ex; status[3] as there. smpq_pack_weights_s2d = the same with step NULL.
 * smpq_stem_conv_s2d_q: as smpq_conv2d_fwd_q with the stem geometry (h, w = the ORIGINAL image
 *   size; output [n][ceil(h/2)][ceil(w/2)][cout] NHWC), no residual; cout % 16 == 0; tile_cfg one
 *   of the tile configs with 64 output channels per block, or -1. */
int smpq_image_quantize_s2d(const float* x, int n, int c, int h, int w, const float* absmax, int limbs,
                            int8_t* out, smpq_stream_t stream);
int smpq_pack_weights_s2d_ex(const float* w, int cout, int cin, const float* step, int wlimbs, int8_t* codes,
                             float* wscale, int32_t* status, smpq_stream_t stream);
int smpq_pack_weights_s2d(const float* w, int cout, int cin, int wlimbs, int8_t* codes, float* wscale,
                          int32_t* status, smpq_stream_t stream);
int smpq_stem_conv_s2d_q(const int8_t* xq, const float* x_absmax, int n, int h, int w, const int8_t* codes,
                         int wlimbs, int cout, const float* col_scale, const float* col_shift, int relu,
                         int limbs, float* y, float* y_absmax, int8_t* yq, float yq_range, int32_t* overflow,
                         int tile_cfg, smpq_stream_t stream);

/* Fused stem, static-range mode: conv1 7x7/2/3 + bn1 + ReLU + maxpool 3x3/2/1 (resnet.py:143-147,
 * ResNet.forward resnet.py:206-209) in one launch, on smpq_image_quantize_s2d planes and
 * smpq_pack_weights_s2d codes -> the POOLED output's limb planes yq [limbs][n][h/4][w/4][64]
 * (h, w = the original image size). Bitwise identical to smpq_stem_conv_s2d_q (relu = 1, yq with
 * the same range, y = NULL) followed by smpq_maxpool_limbs; *overflow is set to 1 when a conv
 * output exceeded the range (then clamped). smpq_stem_pool_supported returns 1 for the shapes it
 * handles: cout == 64, h and w multiples of 4, w <= 224, (limbs, wlimbs) in {(3,3), (2,2), (1,2)};
 * otherwise use the two-launch path. */
int smpq_stem_pool_supported(int n, int h, int w, int cout, int limbs, int wlimbs);
int smpq_stem_pool_s2d_q(const int8_t* xq, const float* x_absmax, int n, int h, int w, const int8_t* codes,
                         int wlimbs, int cout, const float* col_scale, const float* col_shift, int limbs,
                         int8_t* yq, float yq_range, int32_t* overflow, smpq_stream_t stream);

/* AdaptiveAvgPool2d(1) + flatten + fc (ResNet._forward_impl resnet.py:216-218; modules built at
 * resnet.py:162-163) on the last block's NHWC fp32 output x [n][hw][c]: pooled[n][c] = (sum over
 * the hw pixels in order) * (1 / hw), logits[n][nout] = pooled . fc_w[nout][c] (+ fc_b[nout]),
 * summed over c in order with fused multiply-adds. Every logit is computed in an order that does
 * not depend on n or on the other images, so an image's logits are the same bits whatever batch
 * or data-parallel shard it runs in. pooled_ws: device fp32 [n][c] (workspace, holds the pooled
 * features afterwards); fc_b may be NULL; c % 4 == 0. */
int smpq_avgpool_fc(const float* x, int n, int hw, int c, const float* fc_w, const float* fc_b, int nout,
                    float* pooled_ws, float* logits, smpq_stream_t stream);

/* Tile configurations of smpq_conv2d_fwd (for autotuning): count, and BM (pixels) x BN (output
 * channels) / threads. Every configuration gives bitwise-identical results. */
int smpq_conv2d_num_tile_configs(void);
int smpq_conv2d_tile_config(int cfg, int* bm, int* bn, int* threads);

/* Kernel family of a tile configuration:
 *   SMPQ_TILE_LDS_DMA          LDS-DMA loader; cin % 64 == 0, cout % 16 == 0, every operand and
 *                              output plane < 2 GiB
 *   SMPQ_TILE_LDS_DMA_K128     as SMPQ_TILE_LDS_DMA with 128-wide K steps: also cin % 128 == 0
 *   SMPQ_TILE_HALO3X3          (ABI 5) halo-patch 3x3 kernel: 3x3 / stride 1 / pad 1 convs with
 *                              cin % 64 == 0, cout % 64 == 0, one weight limb, 2 or 3 activation
 *                              limbs, static-range limb-plane output with ReLU (yq set,
 *                              relu != 0; y, y_absmax, residual NULL), optionally with a
 *                              limb-plane residual_q (round 6) — other calls return
 *                              SMPQ_E_INVALID.
 *                              Its configurations follow the LDS-DMA ones; BM = the tile's pixels
 *                              (TH x TW of one image), BN = 64.
 *   SMPQ_TILE_RESIDENT1X1      (ABI 6) weight-stationary 1x1 tiles: 1x1 / pad 0 convs with cin
 *                              64 .. 1024 (per configuration: smpq_conv2d_tile_supported), cout a
 *                              multiple of the slab (BN = 64 / 128 / 256), 3 activation limbs,
 *                              static-range limb-plane output (yq set; y, y_absmax, residual NULL);
 *                              3 weight limbs without ReLU or residual_q (the downsamples), 1 weight
 *                              limb with ReLU and optionally residual_q (both with or without weight
 *                              offsets), or neither (no offsets) — other calls return
 *                              SMPQ_E_INVALID. A persistent workgroup keeps its slab's weight limbs
 *                              in registers and walks pixel tiles; BM = pixels per tile, BN = the
 *                              slab. Configurations follow the halo ones.
 * (negative: error code). Values 0 and 1 were the register-staged family (ABI <= 3, removed). */
#define SMPQ_TILE_LDS_DMA 2
#define SMPQ_TILE_LDS_DMA_K128 3
#define SMPQ_TILE_HALO3X3 4
#define SMPQ_TILE_RESIDENT1X1 5
int smpq_conv2d_tile_kind(int cfg);

/* 1 if tile configuration cfg can run a conv of this shape and these limb counts (the rules the
 * launch applies: loader family, K-step width, accumulator budget, LDS per CU), else 0. Every
 * supported configuration gives bitwise-identical results. */
int smpq_conv2d_tile_supported(int cfg, int cin, int cout, int kh, int kw, int limbs, int wlimbs);

/* Workspace the conv needs (none today; kept for ABI stability). */
size_t smpq_conv2d_workspace_bytes(int n, int h, int w, int cin, int cout, int kh, int kw,
                                   int stride, int pad, int limbs);

/* ---- evaluation reductions (functions.py:84-149) ---------------------------------------------
 * smpq_softmax_xent: one batch of logits [rows][cols] fp32 with int64 labels [rows]:
 *   probs  fp32 [rows][cols] softmax = exp(x - max) / sum (functions.py:117), or NULL
 *   stats  double [4], ACCUMULATED (+=): [0] batch-mean cross entropy (criterion(output, y),
 *          :116 — one term per call, as loss_sum += loss at :121), [1] rows whose first maximal
 *          class equals the label (output.max(1), :114), [2] rows, [3] batches (+1)
 *   row_ws fp32 workspace [2 * rows]
 * smpq_kl_rows: stats double [2] += {sum over rows of sum_c p_ref * log(p_ref / p), rows}
 *   (functions.py:140-146; KLdiv = stats[0] / stats[1]); row_ws fp32 [rows].
 * Rows are reduced in a fixed order in double: results do not depend on launch timing. A label
 * outside [0, cols) makes that row's loss NaN (the reference raises). */
int smpq_softmax_xent(const float* logits, const int64_t* labels, int rows, int cols, float* probs,
                      double* stats, float* row_ws, smpq_stream_t stream);
int smpq_kl_rows(const float* p_ref, const float* p, int rows, int cols, double* stats, float* row_ws,
                 smpq_stream_t stream);

/* ---- content fingerprints (cache validation; smpq/engine.py) ------------------------------------
 * smpq_fingerprint: out[t] = sum_i H(w_i, i) mod 2^64 over the ceil(nbytes[t] / 4) 32-bit words of
 *   tensor t (device pointers ptrs[t], 4-B aligned, a device array; a partial last word is
 *   zero-padded), for t < ntensors; the work is split into
 *   nchunks chunks of smpq_fingerprint_chunk_words() words: chunk c covers tensor chunk_tensor[c]
 *   from word chunk_word[c] (device arrays). out (device uint64 [ntensors]) is overwritten.
 *   H(w, i) = fmix32(w ^ i*0x9E3779B9) | fmix32(w ^ (i*0x85EBCA6B + 0xC2B2AE35)) << 32, fmix32 = the
 *   MurmurHash3 finalizer (all arithmetic mod 2^32): injective in w for each i, so any single-word
 *   change changes the fingerprint, and structured multi-word changes cancel with p ~ 2^-64.
 * smpq_fingerprint_compare: *flag |= 1 if a[i] != b[i] for some i < n (device arrays).
 * smpq_fingerprint_host: the same sum over nbytes bytes of host memory.
 * Used to detect in-place writes through `.data` (functions.py:22, resnet50_main.py:191) that
 * leave a Parameter's version counter unchanged. */
long long smpq_fingerprint_chunk_words(void);
int smpq_fingerprint(const void* const* ptrs, const int64_t* nbytes, int ntensors, const int32_t* chunk_tensor,
                     const int64_t* chunk_word, int nchunks, uint64_t* out, smpq_stream_t stream);
int smpq_fingerprint_compare(const uint64_t* a, const uint64_t* b, int n, int32_t* flag, smpq_stream_t stream);
uint64_t smpq_fingerprint_host(const void* p, int64_t nbytes);

/* Diagnostics: one v_mfma_i32_16x16x64_i8 with the kernel's fragment mapping.
 *   a [16][64] int8 row-major, b [16][64] int8 (b[col][k]), c [16][16] int32 row-major */
int smpq_debug_mfma_i8(const int8_t* a, const int8_t* b, int32_t* c, smpq_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* SMPQ_H_ */
