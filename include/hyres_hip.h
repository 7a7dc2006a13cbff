/*
 * hyres_hip.h — C-ABI of libhyres_hip.so, the MI355X (gfx950) kernels behind HyRES's
 * residual-codec hot path.  Plain pointers and sizes only: every tensor argument is a device
 * pointer to fp32 data laid out NHWC ([B][H][W][ld] with the channel slice starting at the
 * pointer), every entry point takes the caller's HIP stream as an opaque handle and returns
 * 0 on success or a nonzero HYRES_E_* / hipError_t code (message: hyres_last_error_string()).
 * The library never allocates, frees or synchronises: scratch is caller-supplied (query with the
 * *_workspace_bytes functions), so every call is stream-ordered and hipGraph-capturable.
 *
 * The reference has no native operator API — its "operator interface" is nn.Module.forward +
 * autograd.  Each entry point below names the reference code it replaces
 * (paths relative to the reference repo root).
 */
#ifndef HYRES_HIP_H
#define HYRES_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

typedef void* hyres_stream_t; /* hipStream_t */

#define HYRES_OK 0
#define HYRES_E_SHAPE 1001     /* inconsistent or unsupported shape / stride */
#define HYRES_E_ALIGN 1002     /* pointer or leading dimension not 16-byte aligned where needed */
#define HYRES_E_ARG 1003       /* invalid enum / NULL pointer */
#define HYRES_E_WORKSPACE 1004 /* workspace too small */

#define HYRES_MAX_TAPS 49

/* ------------------------------------------------------------------------------------------ */
/* library                                                                                    */
/* ------------------------------------------------------------------------------------------ */
int hyres_version(void);
const char* hyres_last_error_string(void);


/* ------------------------------------------------------------------------------------------ */
/* convolution geometry (implicit GEMM, NHWC).                                                */
/* One launch computes Y[b, i*osh+oph[p], j*osw+opw[p], co] for every phase p < nphase and base */
/* pixel (i,j) < (Hq,Wq):  bias[co] + sum over taps t of phase p and ci < Ci of                 */
/*   X[b, i*ish + dh[t], j*isw + dw[t], ci] * W2[co*ldw + t*Ci + ci]   (zero outside X).        */
/* Phases express ConvTranspose2d / strided-conv input-gradients as sub-pixel convolutions.    */
/* ------------------------------------------------------------------------------------------ */
typedef struct hyres_conv_geom {
    int B, Hi, Wi, Ci, ldx;   /* input: NHWC, pixel stride ldx floats */
    int Ho, Wo, Co, ldy;      /* output tensor dims, pixel stride ldy floats */
    int nphase, Hq, Wq;       /* base grid per phase */
    int osh, osw, ish, isw;   /* output / input stride of the base grid */
    int oph[4], opw[4];       /* output offset of each phase */
    int ntap[4], tap0[4];     /* taps of each phase: global tap indices tap0[p] .. tap0[p]+ntap[p]-1 */
    int ntaps;                /* total taps (rows of W2 = ntaps*Ci per output channel) */
    int dh[HYRES_MAX_TAPS], dw[HYRES_MAX_TAPS];
    int kh[HYRES_MAX_TAPS], kw[HYRES_MAX_TAPS]; /* kernel element each tap reads (weight re-layout) */
} hyres_conv_geom;

/* Keep only the taps whose kernel element (kh, kw) has keep[kh*KW + kw] != 0 (order preserved).
 * CheckboardMaskedConv2d's forward/dgrad run on its 12 live taps of 25. */
int hyres_geom_filter_taps(hyres_conv_geom* g, const unsigned char* keep, int KW);

/* nn.Conv2d(k, stride, pad, dil) forward (models/layers/common.py:4-11, compressai conv()). */
int hyres_geom_conv2d(hyres_conv_geom* g, int B, int H, int W, int Ci, int ldx, int Co, int ldy,
                      int KH, int KW, int stride, int pad, int dil);
/* input-gradient of that Conv2d: a conv over dY (stride 1) or a 4-phase sub-pixel conv (stride 2).
 * (B,H,W,Ci,Co,...) describe the ORIGINAL conv; ld_dx / ld_dy are the gradients' pixel strides. */
int hyres_geom_conv2d_dgrad(hyres_conv_geom* g, int B, int H, int W, int Ci, int ld_dx, int Co,
                            int ld_dy, int KH, int KW, int stride, int pad, int dil);
/* nn.ConvTranspose2d(k, s=2, p, output_padding=1) forward (compressai deconv()) as 4 phases. */
int hyres_geom_deconv2d(hyres_conv_geom* g, int B, int H, int W, int Ci, int ldx, int Co, int ldy,
                        int K, int pad);
/* input-gradient of that ConvTranspose2d: a stride-2 conv over dY. */
int hyres_geom_deconv2d_dgrad(hyres_conv_geom* g, int B, int H, int W, int Ci, int ld_dx, int Co,
                              int ld_dy, int K, int pad);

/* Weight re-layout for a geometry built by the helpers above.  ``w`` is the PyTorch parameter
 * (Conv2d: [Co][Ci][KH][KW]; ConvTranspose2d: [Ci][Co][K][K]); ``w2`` gets [rows][ntaps*cols] in
 * the geometry's tap order.  ``mask`` (same shape as w, or NULL) multiplies w on the fly
 * (CheckboardMaskedConv2d, models/layers/checkerboard.py:46-47). (Ci, Co) are the ORIGINAL layer's. */
#define HYRES_WPREP_CONV 0        /* Conv2d forward:  rows = Co, cols = Ci */
#define HYRES_WPREP_CONV_DGRAD 1  /* Conv2d dgrad:    rows = Ci, cols = Co, taps flipped as geom */
#define HYRES_WPREP_DECONV 2      /* ConvT forward:   rows = Co, cols = Ci, phase tap order */
#define HYRES_WPREP_DECONV_DGRAD 3/* ConvT dgrad:     rows = Ci(in), cols = Co(out) */
int hyres_conv_weight_prep(const hyres_conv_geom* g, const float* w, float* w2, int mode, int Ci,
                           int Co, int KH, int KW, int pad, const float* mask, hyres_stream_t s);
/* Batched re-layout: every conv weight of a model in ONE launch per optimiser step.
 * hyres_prep_desc_fill writes one descriptor (hyres_prep_desc_bytes() bytes, host memory) for the same
 * arguments as hyres_conv_weight_prep, covering output elements [begin, begin + rows*ntaps*cols);
 * hyres_conv_weight_prep_batch runs n device-resident descriptors (sorted by begin, total elements). */
long long hyres_prep_desc_bytes(void);
int hyres_prep_desc_fill(void* desc, const hyres_conv_geom* g, const float* w, float* w2, int mode, int Ci, int Co,
                         int KH, int KW, long long begin, long long* count);
int hyres_conv_weight_prep_batch(const void* descs, int n, long long total, hyres_stream_t s);

/* epilogue of the convolution GEMM */
#define HYRES_EPI_BIAS 0      /* y = act(acc + bias + res) */
#define HYRES_EPI_GDN 1       /* n = acc + bias(beta');  y = aux0 * rsqrt(n); out2 = n   (GDN)  */
#define HYRES_EPI_IGDN 2      /* n = acc + bias(beta');  y = aux0 * sqrt(n);  out2 = n   (IGDN) */
#define HYRES_EPI_GDN_BWD 3   /* y = 2*aux0*acc + aux1 * rsqrt(aux2)                              */
#define HYRES_EPI_IGDN_BWD 4  /* y = 2*aux0*acc + aux1 * sqrt(aux2)                               */
#define HYRES_EPI_ROWSCALE 5  /* y = act(aux1[pix * ld1] * acc + bias (+ res)): a per-output-pixel scale of the
                               * input folded into the GEMM (SpatialAttention's x * attn ahead of MultiScaleRefine's
                               * fusion 1x1, enhancement.py:105-109)                                          */
#define HYRES_EPI_SA_BWD 6    /* y = acc + aux0[pix * ld0] + (n == ((const int*)aux2)[pix] ? aux0[pix * ld0 + 1] : 0):
                               * SpatialAttention's channel-mean / channel-max backward (enhancement.py:14-20)
                               * folded into the input-gradient of MultiScaleRefine's fusion 1x1 (training with
                               * the ROWSCALE forward): aux0 = [P][2] (d mean / C, d max), aux2 = argmax [P]  */
#define HYRES_ACT_NONE 0
#define HYRES_ACT_RELU 1
#define HYRES_ACT_PRELU 2     /* single shared slope (nn.PReLU()), read from device pointer */
#define HYRES_ACT_RELU_MASK 3 /* ReLU backward fused into an input-gradient: y = (aux0 > 0) ? y : 0,
                                 aux0 = the ReLU output of the layer whose gradient is produced */
#define HYRES_ACT_PRELU_MASK 4 /* PReLU backward fused into an input-gradient (round 6; the 3x3 Ci = Co = 64 layers on
                                * conv3x3_wres_bf6_kernel only, HYRES_E_ARG elsewhere): y = (aux0 > 0) ? v : slope[0] * v,
                                * aux0 = the saved pre-activation (fp32, pitch ld0), and the slope gradient
                                * sum_{aux0 <= 0} aux0 * v is ADDED to ((float*)aux1)[0] — per-block partials in aux2
                                * (capacity ld2 floats >= HYRES_PRELU_PARTIALS), summed in a fixed order by a second
                                * kernel of the same call (deterministic). kind BIAS, accumulate 0, fp32 IO.
                                * Replaces prelu_bwd of MultiScaleRefine's scale blocks (enhancement.py:44-51,
                                * 89-95): the dilation-2 conv's input-gradient writes the PReLU'd gradient directly.
                                * With kind HYRES_EPI_SA_BWD (round 6, the streaming 64 -> 192 input-gradients only):
                                * output channels [0, 64) get the PReLU backward — aux1 = their pre-activation (Y's
                                * dtype, pitch ld1), slope gradient ADDED to ((float*)res)[0], partials in out2
                                * (ldo2 >= HYRES_PRELU_PARTIALS); no accumulate. Replaces MultiScaleRefine scale 1's
                                * prelu_bwd (its PReLU output is multi[..., 0:64], enhancement.py:113-115) */
#define HYRES_PRELU_PARTIALS 2048

#define HYRES_IO_X16 1   /* hyres_epilogue.io_f16 bits */
#define HYRES_IO_Y16 2
#define HYRES_IO_AUX16 4
typedef struct hyres_epilogue {
    int kind, act, accumulate;    /* accumulate: y += result (gradient accumulation) */
    int square_input;             /* GEMM A-operand prologue x -> x*x (GDN norm) */
    const float* bias;            /* [Co] or NULL */
    const float* res; int ldres;  /* added before act, or NULL */
    const float* slope;           /* PReLU slope (device, 1 float) */
    const float* aux0; int ld0;
    const float* aux1; int ld1;
    const float* aux2; int ld2;
    float* out2; int ldo2;
    int f16_operands;             /* 1: X and W2 rounded to fp16 in the LDS staging, v_mfma_f32_32x32x16_f16
                                   * with fp32 accumulation and fp32 epilogue (autocast-fp16 inference,
                                   * BASELINE configs[4]); ignored on the small-Ci and narrow paths */
    int io_f16;                   /* fp16 activations in HBM (autocast, configs[4] and AMP training): bit 0 =
                                   * X is fp16, bit 1 = Y and the epilogue's activation operands (res, aux0,
                                   * out2) are fp16 (bias/slope stay fp32); bits 0/1: no accumulate, no
                                   * GDN-backward kinds. X-fp16 needs Ci % 32 == 0 (or the narrow Co <= 4
                                   * kernel, whose Y stays fp32). Bit 2 (HYRES_IO_AUX16, backward convs with
                                   * fp32 X/Y): the saved activations the epilogue reads — aux0 (the ReLU
                                   * mask's y, GDN-backward's x) and aux2 (GDN-backward's norm) — are fp16. */
} hyres_epilogue;

/* Y = conv(X, W2) with the epilogue — nn.Conv2d / nn.ConvTranspose2d / GDN forward and their
 * input-gradients (replaces torch's cuDNN/MIOpen conv dispatch at every conv call site on the hot
 * path: models/checkerboard.py:35-88, models/layers/attention.py:11-39,
 * models/layers/enhancement.py:17,44-51,65-82, compressai GDN/RBB).  fp32 MFMA (v_mfma_f32_32x32x2f32). */
int hyres_conv_forward(const hyres_conv_geom* g, const float* x, const float* w2, int ldw, float* y,
                       const hyres_epilogue* e, void* workspace, long long ws_bytes, hyres_stream_t s);
/* Scratch for split-K on small-M layers (0 = none needed).  Passing a NULL / short workspace is
 * valid: the launch then runs unsplit (same result, fewer blocks in flight). */
long long hyres_conv_workspace_bytes(const hyres_conv_geom* g);
/* Name of the kernel hyres_conv_forward launches for (g, e) — split != 0 when a workspace of
 * hyres_conv_workspace_bytes(g) is passed — as rocprof prints it, e.g.
 * "conv_fwd_kernel<2, 1, 2, 2, 0, false, false>" (16B-aligned operands assumed).  Host-only, no
 * launch: the profiling label of bench.py's roofline line comes from the launcher's own choice. */
int hyres_conv_kernel_name(const hyres_conv_geom* g, const hyres_epilogue* e, int split, char* buf, int n);
/* Tuning override of the conv planners (sweeps only; not used by the product path). key 0: tile
 * (0 = 128x128, 1 = 128x64, 2 = 128x32, 3 = 64x128, 4 = 64x64), 1: split-K target block count,
 * 2: minimum K chunks per split; value -1 restores the built-in heuristic. *old (may be NULL) gets the
 * previous value. Not thread-safe against concurrent launches. */
/* The launcher's choice for (g, e): *tile = 0..4 as above (-1: the narrow VALU kernel), *nsplit = split-K
 * factor (1 = fused epilogue). Pure host function. */
int hyres_conv_plan(const hyres_conv_geom* g, const hyres_epilogue* e, int* tile, int* nsplit);
#define HYRES_TUNE_TILE 0
#define HYRES_TUNE_SPLIT_BLOCKS 1
#define HYRES_TUNE_SPLIT_MINCHUNKS 2
#define HYRES_TUNE_WGRAD_BLOCKS 3     /* weight gradients: split-K target block count */
#define HYRES_TUNE_WGRAD_MINCHUNKS 4  /* minimum 32-pixel chunks per split */
#define HYRES_TUNE_WGRAD_NT 5         /* 1: no tap grouping (one tap per block column group) */
#define HYRES_TUNE_WGRAD_MAXSPLIT 6   /* maximum split count (default 256; 64 on <= 16384-pixel grids) */
#define HYRES_TUNE_F32_GEMM 7         /* GEMM of the fp32 convolutions (forward, input-gradient, and the halo-staged /
                                       * 1x1 weight gradients): 1 bf16x6 (default: each fp32 operand split into 3 bf16
                                       * pieces, the 6 cross products with i + j <= 2, fp32 accumulation — per-product
                                       * error <= ~2^-25, i.e. fp32-accurate, on the 16x faster bf16 MFMA; DESIGN §4
                                       * "bf16x6"), 0 the native fp32 MFMA */
#define HYRES_TUNE_STREAM_H 8         /* 1 (default): fp16-activation 1x1 convs with K, Co <= 128 on >= 16384 pixels on the
                                       * streaming kernel (conv1x1_stream_h_kernel); 0: the tiled kernel (A/B) */
#define HYRES_TUNE_WRES_BF6_GUARD 9   /* 1 (default): the bf16x6 weight-resident 3x3 conv and the fused f16 ResidualUnit declare the whole VGPR file of
                                       * its SIMDs, so no other kernel's wave shares them; 0: DIAGNOSTIC ONLY, the
                                       * allocation under which co-resident waves computed wrong values (DESIGN §4
                                       * "Cross-kernel interference") */
#define HYRES_TUNE_STREAM_B6 10       /* 1 (default): the fp32 1x1 convs with (Ci, Co) in {(64,64), (64,128), (128,64)} on
                                       * >= 65536 pixels on the bf16x6 streaming kernel (conv1x1_stream_b6_kernel, any of
                                       * residual / ReLU mask / accumulate); 0: the tiled implicit GEMM (A/B) */
#define HYRES_TUNE_STREAM_CE 11       /* 1 (default): conv1x1_stream_b6_kernel stages each co tile's accumulator through LDS
                                       * so its epilogue reads / writes whole 128-byte pixel-row pieces; 0: the MFMA
                                       * lane layout straight to HBM (32 B per pixel row per wave instruction; A/B) */
#define HYRES_TUNE_WRES_BF6_V 12      /* conv3x3_wres_bf6_kernel variant: bit 0 (default 1) each tap's fragments read
                                       * one tap ahead, bit 1 static priority 1 for waves 4..7; 0: reads as the compiler
                                       * schedules them (A/B) */
#define HYRES_TUNE_NARROW_STRIP 13    /* 1 (default): Co <= 4 convs whose phases' taps are <= 3x3 grids, Wq % 4 == 0, on
                                       * conv_narrow_strip_kernel (4-pixel strips, weights in VGPRs); 0: conv_narrow_kernel */
#define HYRES_TUNE_WRES32 14          /* 1 (default): fp32 3x3 Ci = 64 convs on the weight-resident kernels
                                       * (conv3x3_wres_bf6 / _f32); 0: the implicit GEMM (A/B) */
#define HYRES_TUNE_WGRAD_PF 15        /* bf16x6 1x1 weight gradients: 2 (default) = operand loads two chunks ahead
                                       * (wgrad1x1_bf6_pf2_kernel), 1 = one chunk ahead (wgrad1x1_bf6_kernel) */
#define HYRES_TUNE_WGRAD_HALO_PF 16   /* bf16x6 3x3 halo weight gradients (one kernel row of 3 taps per block): 2
                                       * (default) = operand loads two chunks ahead (wgrad_halo_bf6_pf2_kernel), 1 = one
                                       * chunk ahead; the 5x5s stay on wgrad_halo_bf6_kernel (slower two ahead) */
#define HYRES_TUNE_STREAM_HF 17       /* 1 (default): fp16-IO 1x1 convs (Ci, Co in {64, 128}, >= 16384 px) with a residual /
                                       * ReLU-mask / accumulate operand on conv1x1_stream_hf_kernel; 0: the f16 tiles */
#define HYRES_TUNE_SMALL_TILE 18      /* 1 (default): fp32 implicit-GEMM tiles on <= 65536-pixel grids by the round-6 rule
                                       * (64x64 for the short-K 1x1s with Co <= 192, 128x128 for Co >= 512;
                                       * profiles/r6g_tile32.txt); 0: the round-5 rule (A/B) */
#define HYRES_TUNE_B6_SWIZZLE 19      /* 1 (default): the bf16x6 implicit GEMM stages its split planes in 64-B LDS rows with the
                                       * 16-B slots XOR-swizzled by row (conflict-free stores and reads); 0: 80-B padded rows
                                       * (2-way store conflicts), A/B; bit-identical */
#define HYRES_TUNE_B6_DB 20           /* the bf16x6 implicit GEMM's 64x64 tile staging K chunks in two LDS buffers (one barrier
                                       * per chunk, conv_fwd_b6db_kernel): 1 always, -1 on grids of <= 16384 output pixels,
                                       * 0 (default) never (one buffer, two barriers; faster in the graphed step); bit-identical */
#define HYRES_TUNE_STREAM_SAB 21      /* 1 (default): the SA_BWD input-gradient of MultiScaleRefine's fusion 1x1 (64 -> 192 on
                                       * >= 65536 pixels) on conv1x1_stream_b6_kernel<6, 4, 8 | acc>, its ROWSCALE forward
                                       * (192 -> 64) on <2, 12, 16>, and under AMP the SA_BWD input-gradient on
                                       * conv1x1_stream_hf_kernel<6, 4, 8 | acc>; 0: the implicit GEMMs */
#define HYRES_TUNE_WGRAD_HALO5_PF 22  /* 1: the 5-tap-row halo weight gradients (5x5, stride 1 / 2) also on the two-chunks-
                                       * ahead kernel (with key 16 = 2; bit-identical); 0 (default): one chunk ahead — no
                                       * gain per launch or in the step (profiles/r6v_wg5.txt, r6v_wg5_step_ab.txt) */
#define HYRES_TUNE_THIN_WINDOW 23     /* 1 (default): the thin (3-channel) 3x3 weight gradients keep each pixel's 3 x 3 Q window
                                       * in registers, sliding one column per pixel (bit-identical); 0: nine LDS reads per pixel */
#define HYRES_TUNE_KEYS 24
int hyres_conv_tuning(int key, int value, int* old);

/* Weight gradient:  dW[t][m][n] = sum_q P[q][m] * Q[shift_t(q)][n]  over a base grid q (B,Hq,Wq).
 * Conv2d: P = dY (output grid), Q = X;  ConvTranspose2d: P = X (input grid), Q = dY.
 * Result written (or accumulated) into the PyTorch-layout gradient dst[m*sm + n*sn + t*st]. */
typedef struct hyres_wgrad_desc {
    int B, Hq, Wq;               /* base grid (P's pixel grid) */
    int M, ldp;                  /* P channels / pixel stride */
    int N, ldq, Hqq, Wqq;        /* Q channels / pixel stride / Q spatial dims */
    int sq;                      /* Q stride of the base grid */
    int ntaps;
    int dh[HYRES_MAX_TAPS], dw[HYRES_MAX_TAPS];
    int sm, sn, st;              /* destination strides (floats) */
    int square_q;                /* Q -> Q*Q (GDN gamma gradient) */
    int accumulate;
    int f16_operands;            /* AMP: P, Q rounded to fp16 on the f16 MFMA, fp32 accumulation */
    int io_f16;                  /* fp16 operands in HBM (AMP training, fp16 saved activations): bit 0 = P is
                                  * fp16, bit 1 = Q is fp16; read natively by the f16 weight-gradient kernels
                                  * and the thin kernel (P), converted to fp32 scratch for the others */
} hyres_wgrad_desc;
int hyres_wgrad_desc_conv2d(hyres_wgrad_desc* d, int B, int H, int W, int Ci, int ldx, int Co,
                            int ldy, int KH, int KW, int stride, int pad, int dil);
int hyres_wgrad_desc_deconv2d(hyres_wgrad_desc* d, int B, int H, int W, int Ci, int ldx, int Co,
                              int ldy, int K, int pad);
long long hyres_wgrad_workspace_bytes(const hyres_wgrad_desc* d);
/* dbias (optional, may be NULL): dbias[m] (+)= sum_q P[q][m] — the Conv2d bias gradient when P = dY
 * (replaces the separate colsum for conv layers; fused into the weight-gradient kernel). */
int hyres_conv_wgrad(const hyres_wgrad_desc* d, const float* p, const float* q, float* dst,
                     float* dbias, void* workspace, long long ws_bytes, hyres_stream_t s);

/* Deferred split-K reduce (same reference operation as hyres_conv_wgrad: the weight / bias gradient of
 * one conv in loss.backward(), src/utils/engine.py:63 via models/checkerboard.py:35-88). A weight
 * gradient is a GEMM over the batch's pixels, split over pixel ranges into [nsplit][ntaps][M][N]
 * partial slabs; hyres_conv_wgrad reduces them with one launch per layer. The deferred form launches
 * only the GEMM kernel and returns the reduce as up to two jobs (weight, then bias); the caller keeps
 * the workspace untouched and the destinations unread until hyres_wgrad_reduce_jobs has run them on the
 * same stream, where one launch reduces up to HYRES_WGRAD_MAX_JOBS jobs (a gradient segment of many
 * layers). Jobs of one launch must not write overlapping destinations. The result is bit-identical to
 * hyres_conv_wgrad's (same split plan, same per-output summation order). */
#define HYRES_WGRAD_MAX_JOBS 48
typedef struct hyres_wgrad_job {
    const float* slab;   /* [nsplit][ntaps][M][N] partials in the workspace */
    float* dst;          /* dst[m*sm + n*sn + t*st] (+)= sum over the nsplit partials */
    int nsplit, ntaps, M, N;
    int sm, sn, st, accumulate;
    int lanes;           /* reduce layout the launcher chose (4, 8 or 16): fixes the summation order */
    int reserved;
} hyres_wgrad_job;
int hyres_conv_wgrad_deferred(const hyres_wgrad_desc* d, const float* p, const float* q, float* dst,
                              float* dbias, void* workspace, long long ws_bytes, hyres_wgrad_job* jobs,
                              int* njobs, hyres_stream_t s);
int hyres_wgrad_reduce_jobs(const hyres_wgrad_job* jobs, int n, hyres_stream_t s);

/* Fused ResidualUnit / ResidualBottleneckBlock forward, autocast inference with fp16 activations (round 4):
 * y = [relu](x + W3 * relu(W2 (*) relu(W1 * x + b1) + b2) + b3) in ONE launch, t1 / t2 kept on chip (fp16, the
 * unfused path's rounding points). Replaces the three-conv chain of the ResidualUnit in models/layers/attention.py:11-30
 * (final_relu = 1) and of compressai's ResidualBottleneckBlock at models/checkerboard.py:38,42,51,56 (final_relu = 0).
 * x, y: [B][H][W][N] fp16, N = 128, W % 64 == 0 (hyres_ru_fused_f16_ok); weights / biases fp32 in the PyTorch
 * layouts (w1 [N/2][N], w2 [N/2][N/2][3][3], w3 [N][N/2]), converted to fp16 on load; 16-byte aligned. */
int hyres_ru_fused_f16_ok(int B, int H, int W, int N);
int hyres_ru_fused_f16(const void* x, void* y, int B, int H, int W, int N, const float* w1, const float* b1,
                       const float* w2, const float* b2, const float* w3, const float* b3, int final_relu,
                       void* t1, void* t2, hyres_stream_t s);
/* t1, t2: NULL (inference), or [B][H][W][N/2] fp16 outputs receiving the two intermediates (AMP training: the
 * backward of the three convs reads them). */

/* column sums over pixels: dst[c] (+)= sum_p x[p*ld + c]  (bias gradients) */
int hyres_colsum(const float* x, int P, int C, int ld, float* dst, int accumulate, void* workspace,
                 long long ws_bytes, hyres_stream_t s);
long long hyres_colsum_workspace_bytes(int P, int C);
/* the same over a fp16 x (AMP fp16 gradients), fp32 sums */
int hyres_colsum_f16(const void* x, int P, int C, int ld, float* dst, int accumulate, void* workspace,
                     long long ws_bytes, hyres_stream_t s);

/* ------------------------------------------------------------------------------------------ */
/* layout / elementwise                                                                       */
/* ------------------------------------------------------------------------------------------ */
int hyres_nchw_to_nhwc(const float* x, float* y, int B, int C, int H, int W, int ldy, hyres_stream_t s);
int hyres_nhwc_to_nchw(const float* x, int ldx, float* y, int B, int C, int H, int W, hyres_stream_t s);
/* y = a + alpha*b over n contiguous floats (hyres.py:48,62 glue) */
int hyres_axpby(const float* a, const float* b, float alpha, float* y, long long n, hyres_stream_t s);
/* x_hat = clamp(x0 + r, 0, 1)  (models/hyres.py:66-67); bwd: g passes where 0 < x0+r < 1 */
int hyres_add_clamp01(const float* x0, const float* r, float* y, long long n, hyres_stream_t s);
int hyres_add_clamp01_bwd(const float* pre, const float* g, float* gx, int accumulate, long long n,
                          hyres_stream_t s);
/* g_out = g * (y > 0)   (ReLU backward), optional accumulate into dst */
int hyres_relu_bwd(const float* y, const float* g, float* gx, long long n, hyres_stream_t s);
/* strided variant over NHWC slices */
int hyres_relu_bwd_2d(const float* y, int ldy_, const float* g, int ldg, float* gx, int ldgx, long long P,
                      int C, hyres_stream_t s);
/* PReLU backward from the saved pre-activation x: gx = g*(x>0 ? 1 : a); dslope += sum(g*x*(x<=0))
 * (enhancement.py nn.PReLU). ws: hyres_reduce_workspace_bytes(P*C). */
int hyres_prelu_bwd(const float* x, int ldx, const float* g, int ldg, float* gx, int ldgx, long long P,
                    int C, const float* slope, float* dslope, void* ws, long long ws_bytes,
                    hyres_stream_t s);
/* AttentionBlock gate (models/layers/attention.py:44-47): out = a*sigmoid(b) + x */
int hyres_attn_gate_fwd(const float* a, const float* b, const float* x, float* out, long long n,
                        hyres_stream_t s);
/* fp16 activations (autocast inference): a, b, x, out fp16 in HBM, n % 4 == 0, 8B-aligned. */
int hyres_attn_gate_fwd_f16(const void* a, const void* b, const void* x, void* out, long long n, hyres_stream_t s);
int hyres_attn_gate_bwd(const float* a, const float* b, const float* g, float* ga, float* gb,
                        long long n, hyres_stream_t s);
/* The same with the ReLU backward of a folded in (a = the last ResidualUnit's ReLU output, models/layers/attention.py:
 * 11-30, 44-47): ga = (a > 0) ? g * sigmoid(b) : 0. n % 4 == 0, every operand 16B-aligned (round 6). */
int hyres_attn_gate_bwd_relu(const float* a, const float* b, const float* g, float* ga, float* gb, long long n,
                             hyres_stream_t s);
/* Backward passes with fp16 SAVED activations (AMP training: the forward wrote y / pre / a, b / x / norm as
 * fp16; fp32 arithmetic; 8B-aligned fp16 operands): same semantics as the fp32 entry points of the same name
 * without the suffix. g16 = 1: the gradients in and out (g, gx / ga, gb) are fp16 as well — autocast's own
 * semantics inside the f16 region (the gradient of an fp16 tensor is fp16, src/utils/engine.py:32,50-53);
 * g16 = 0: fp32 gradients. */
int hyres_relu_bwd_2d_f16(const void* y, int ldy_, const void* g, int ldg, void* gx, int ldgx, long long P,
                          int C, int g16, hyres_stream_t s);
int hyres_prelu_bwd_f16(const void* x, int ldx, const void* g, int ldg, void* gx, int ldgx, long long P,
                        int C, const float* slope, float* dslope, void* ws, long long ws_bytes, int g16,
                        hyres_stream_t s);
int hyres_attn_gate_bwd_f16(const void* a, const void* b, const void* g, void* ga, void* gb, long long n, int g16,
                            hyres_stream_t s);
/* ... and with the last ResidualUnit's ReLU backward folded in, as hyres_attn_gate_bwd_relu (round 6); n % 4 == 0,
 * fp16 operands 8B-aligned, fp32 ones 16B-aligned */
int hyres_attn_gate_bwd_relu_f16(const void* a, const void* b, const void* g, void* ga, void* gb, long long n, int g16,
                                 hyres_stream_t s);
/* y (+)= x  (gradient fan-in); _f16: both fp16 */
int hyres_accumulate(const float* x, float* y, long long n, hyres_stream_t s);
int hyres_accumulate_f16(const void* x, void* y, long long n, hyres_stream_t s);
/* y[p*ldy + c] (+)= x[p*ldx + c]  over P pixels x C channels (strided gradient fan-in / copy) */
int hyres_add2d(const float* x, int ldx, float* y, int ldy, long long P, int C, int accumulate,
                hyres_stream_t s);
/* the same with fp16 storage: io bit 0 = x fp16, bit 1 = y fp16 (fp32 add) */
int hyres_add2d_f16(const void* x, int ldx, void* y, int ldy, long long P, int C, int accumulate, int io,
                    hyres_stream_t s);
/* y = a * b elementwise (in-place allowed: CheckboardMaskedConv2d's weight.data *= mask) */
int hyres_mul(const float* a, const float* b, float* y, long long n, hyres_stream_t s);
/* stream-ordered memset 0 (hipMemsetAsync) */
int hyres_zero(void* p, long long bytes, hyres_stream_t s);
/* y (+)= (coef ? coef[0] : 1) * scale * x */
int hyres_scale(const float* x, const float* coef, float scale, float* y, long long n, int accumulate,
                hyres_stream_t s);

/* GDN reparametrisation (compressai NonNegativeParametrizer + LowerBound):
 * beta' = max(beta, bb)^2 - ped,  gamma' = max(gamma, gb)^2 - ped;  and backward. */
int hyres_gdn_reparam_fwd(const float* beta, const float* gamma, float* beta_p, float* gamma_p, int C,
                          hyres_stream_t s);
int hyres_gdn_reparam_bwd(const float* beta, const float* gamma, const float* dbeta_p,
                          const float* dgamma_p, float* dbeta, float* dgamma, int C, int accumulate,
                          hyres_stream_t s);
/* GDN backward helper: dn = g * y / n * (-0.5 GDN | +0.5 IGDN) */
int hyres_gdn_dnorm(const float* g, const float* y, const float* n, float* dn, long long P, int C,
                    int inverse, hyres_stream_t s);
/* the same with fp16 y and n (AMP training); g16: g and dn fp16 too */
int hyres_gdn_dnorm_f16(const void* g, const void* y, const void* n, void* dn, long long P, int C,
                        int inverse, int g16, hyres_stream_t s);

/* ------------------------------------------------------------------------------------------ */
/* quantisation, checkerboard context, entropy models                                         */
/* ------------------------------------------------------------------------------------------ */
/* U(-0.5, 0.5) noise (counter-based hash RNG), replaces torch.empty_like().uniform_() in
 * models/utils/quantization.py:6-10 and compressai EntropyModel.quantize("noise") */
int hyres_uniform_noise(float* out, long long n, unsigned long long seed, unsigned long long offset,
                        hyres_stream_t s);
/* Same distribution with the seed in device memory: draws with seed = mix(*seed_dev ^ salt), then
 * advances *seed_dev (stream-ordered), so a captured HIP graph draws fresh noise on every replay. */
int hyres_uniform_noise_dev(float* out, long long n, unsigned long long* seed_dev, unsigned long long salt,
                            hyres_stream_t s);
/* Quantizer.quantize (models/utils/quantization.py:11-14): mode 0 = "ste" value round(x)-x+x,
 * mode 1 = round (half-to-even) */
int hyres_quantize(const float* x, int mode, float* y, long long n, hyres_stream_t s);
/* Anchor pass (models/checkerboard.py:106-122): y_a = y*[(h+w) even];
 * y_a_hat = STE(y_a - m_a) + m_a  or  y_a + noise. Writes y_a_hat (NHWC [B,H,W,C]). */
int hyres_ckbd_anchor_fwd(const float* y, const float* means_a, int ldm, const float* noise,
                          float* y_a_hat, int B, int H, int W, int C, hyres_stream_t s);
/* Non-anchor pass + combine + GaussianConditional (checkerboard.py:132-142, compressai GC):
 * y_na_hat, y_hat = y_a_hat + y_na_hat, scales = s_a + s_na, means = m_a + m_na,
 * y_q = round(y - means) + means (eval) or y + noise_gc (train), lik = LB(GC(y_q; scales, means)).
 * Also accumulates sum(log lik) per block into ws (bpp partial). */
int hyres_ckbd_nonanchor_gc_fwd(const float* y, const float* y_a_hat, const float* params_a, int lda,
                                const float* params_na, int ldn, const float* noise_q,
                                const float* noise_gc, float* y_hat, float* scales, float* means,
                                float* y_q, float* lik, int B, int H, int W, int C, hyres_stream_t s);
/* backward of the above: g_y = g_yhat (+ GC term in training); [g_scales | g_means] written to
 * both param-aggregation gradient buffers (scales = s_a + s_na, means = m_a + m_na).  The STE /
 * noise quantisers pass the gradient straight to y and give none to the means. */
int hyres_ckbd_gc_bwd(const float* y_q, const float* scales, const float* means, const float* g_lik,
                      const float* g_yhat, int training, float* g_y, float* g_params_a, int lda,
                      float* g_params_na, int ldn, int B, int H, int W, int C, hyres_stream_t s);
/* g_y[anchor positions] += g_ya (context-model path back into the anchor quantiser) */
int hyres_ckbd_anchor_bwd(const float* g_ya, float* g_y, int B, int H, int W, int C, hyres_stream_t s);

/* EntropyBottleneck forward (compressai 1.2.6): z NHWC [P][C]; params packed per channel
 * (see hyres_eb_pack); z_q = z + noise (train) | round(z - med) + med (eval); lik = LB(sig(u)-sig(l));
 * z_hat_ste = quantize_ste(z - med) + med (checkerboard.py:98-101). */
int hyres_eb_fwd(const float* z, const float* packed, const float* noise, int training, float* z_q,
                 float* lik, float* z_hat_ste, long long P, int C, hyres_stream_t s);
int hyres_eb_bwd(const float* z_q, const float* packed, const float* lik, const float* g_lik,
                 const float* g_zhat, int training, int noisequant, float* g_z, float* g_packed_ws,
                 long long P, int C, hyres_stream_t s);
long long hyres_eb_workspace_bytes(long long P, int C);
/* pack EB parameters (softplus(matrices), biases, tanh(factors), quantile medians) per channel */
#define HYRES_EB_REC 64
int hyres_eb_pack(const float* const* mats, const float* const* biases, const float* const* factors,
                  const float* quantiles, float* packed, int C, hyres_stream_t s);
/* reduce the per-block packed gradients of hyres_eb_bwd into the parameter gradients */
int hyres_eb_unpack_grad(const float* g_packed_ws, int nblocks, const float* const* mats,
                         const float* const* factors, float* const* g_mats, float* const* g_biases,
                         float* const* g_factors, float* g_quantiles, int C, int accumulate,
                         hyres_stream_t s);
/* EntropyBottleneck.loss (aux loss) and its gradient wrt quantiles */
int hyres_eb_aux_loss(const float* packed, const float* quantiles, const float* target, float* loss,
                      float* g_quantiles, int C, hyres_stream_t s);

/* ------------------------------------------------------------------------------------------ */
/* MultiScaleRefine pieces (models/layers/enhancement.py)                                     */
/* ------------------------------------------------------------------------------------------ */
/* bilinear, align_corners=False, torch source-index rule (scale = in/out, or 1/scale_factor). */
int hyres_bilinear_fwd(const float* x, int ldx, float* y, int ldy, int B, int Hi, int Wi, int Ho, int Wo,
                       int C, float scale_h, float scale_w, int accumulate, hyres_stream_t s);
int hyres_bilinear_bwd(const float* gy, int ldgy, float* gx, int ldgx, int B, int Hi, int Wi, int Ho,
                       int Wo, int C, float scale_h, float scale_w, int accumulate, hyres_stream_t s);
/* SEBlock (enhancement.py:25-40): s = sigmoid(W2 relu(W1 mean_hw(x))); y = x*s */
int hyres_se_fwd(const float* x, const float* w1, const float* w2, float* y, float* pooled,
                 float* hidden, float* sgate, int B, int HW, int C, int Cr, void* ws, long long ws_bytes,
                 hyres_stream_t s);
int hyres_se_bwd(const float* x, const float* gy, const float* w1, const float* w2,
                 const float* pooled, const float* hidden, const float* sgate, float* gx, float* gw1,
                 float* gw2, int B, int HW, int C, int Cr, void* ws, long long ws_bytes, hyres_stream_t s);
/* hyres_se_bwd with the backward of the PReLU that produced x folded in (round 6; MultiScaleRefine's
 * SE(PReLU(conv_in(x))), enhancement.py:107-110): gx = PReLU'(pre) * dL/dx, the slope gradient
 * sum_{pre <= 0} pre * dL/dx ADDED to dslope[0] (block partials in the workspace, fixed-order sum). fp32; the
 * workspace is hyres_se_workspace_bytes + B*C*4 + 2048*4 bytes. Replaces prelu_bwd after the SE backward. */
int hyres_se_bwd_prelu(const float* x, const float* gy, const float* w1, const float* w2, const float* pooled,
                       const float* hidden, const float* sgate, float* gx, float* gw1, float* gw2, int B, int HW, int C,
                       int Cr, const float* pre, const float* slope, float* dslope, void* ws, long long ws_bytes,
                       hyres_stream_t s);
long long hyres_se_workspace_bytes(int B, int HW, int C);
/* SpatialAttention (enhancement.py:7-21) fused: a = sigmoid(conv7x7([mean_c, max_c])); y = x * a.
 * pooled2 [P][2] and argmax [P] (first maximal channel, torch.max semantics) are saved for backward.
 * C % 4 == 0, 16B-aligned x/y/gy/gx. */
int hyres_spatial_attn_fwd(const float* x, const float* w, float* pooled2, int* argmax, float* attn,
                           float* y, int B, int H, int W, int C, hyres_stream_t s);
int hyres_spatial_attn_bwd(const float* x, const float* w, const float* pooled2, const int* argmax,
                           const float* attn, const float* gy, float* gx, float* gw, int B, int H, int W,
                           int C, void* ws, long long ws_bytes, hyres_stream_t s);
long long hyres_spatial_attn_workspace_bytes(int B, int H, int W);
/* Training with SpatialAttention's multiply folded into MultiScaleRefine's fusion 1x1 (HYRES_EPI_ROWSCALE forward,
 * enhancement.py:105-109): h = PReLU(attn[p] * (W multi)[p] + b), ``pre`` its pre-activation [P][C] (C = fusion
 * width, ldpre), gy = dL/dh [P][ldg]. Writes gs = attn[p] * gp (gp = PReLU-backward of gy: the fusion 1x1's weight-
 * and input-gradient operand), glogit[p] = (1 - attn[p]) * sum_o gp[p,o] * (pre[p,o] - b[o]) (= the gradient at the
 * attention logit: attn * z = pre - b, no division), and ADDS dbias += sum_p gp, dslope += sum_{pre <= 0} gy * pre
 * (deterministic per-block partials). C % 4 == 0, C <= 64, 16B-aligned rows; ws >= hyres_sa_fold_workspace_bytes(P, C). */
long long hyres_sa_fold_workspace_bytes(long long P, int C);
int hyres_sa_fold_bwd(const float* pre, int ldpre, const float* gy, int ldg, const float* attn, const float* bias,
                      const float* slope, float* gs, float* glogit, float* dbias, float* dslope, long long P, int C,
                      void* ws, long long ws_bytes, hyres_stream_t s);
/* ... under AMP training (round 6): ``pre`` fp16 (fp16 activations); g16 = 1: gy and gs fp16 as well (fp16
 * gradients), 0: fp32. fp32 arithmetic; attn, bias, glogit, dbias, dslope fp32. C % 8 == 0, C <= 64, rows 16B-aligned. */
int hyres_sa_fold_bwd_f16(const void* pre, int ldpre, const void* gy, int ldg, const float* attn, const float* bias,
                          const float* slope, void* gs, float* glogit, float* dbias, float* dslope, long long P, int C,
                          void* ws, long long ws_bytes, int g16, hyres_stream_t s);
/* SpatialAttention's map backward from the logit gradient: gw += d conv7x7 weight, gpooled2 = [P][2] gradients of
 * the channel mean (already divided by C, as HYRES_EPI_SA_BWD reads it) and the channel max. ws as
 * hyres_spatial_attn_workspace_bytes(B, H, W). */
int hyres_spatial_attn_bwd_map(const float* glogit, const float* pooled2, const float* w, float* gpooled2, float* gw,
                               int B, int H, int W, int C, void* ws, long long ws_bytes, hyres_stream_t s);
/* fp16-activation forwards (x and y fp16 in HBM, fp32 arithmetic; autocast inference, BASELINE
 * configs[4] "fp16 activations"): same semantics as the fp32 forwards above (bilinear without
 * accumulate; C % 4 == 0, ld % 4 == 0, 8B-aligned x/y). pooled / hidden / sgate / pooled2 / attn fp32. */
int hyres_bilinear_fwd_f16(const void* x, int ldx, void* y, int ldy, int B, int Hi, int Wi, int Ho, int Wo,
                           int C, float scale_h, float scale_w, hyres_stream_t s);
int hyres_se_fwd_f16(const void* x, const float* w1, const float* w2, void* y, float* pooled, float* hidden,
                     float* sgate, int B, int HW, int C, int Cr, void* ws, long long ws_bytes, hyres_stream_t s);
int hyres_spatial_attn_fwd_f16(const void* x, const float* w, float* pooled2, int* argmax, float* attn,
                               void* y, int B, int H, int W, int C, hyres_stream_t s);
/* their backward passes with fp16 x (AMP training); g16 = 1: gy, gx fp16 too (autocast's fp16 activation
 * gradients), g16 = 0: gy, gx fp32. Weight gradients fp32. */
int hyres_se_bwd_f16(const void* x, const void* gy, const float* w1, const float* w2, const float* pooled,
                     const float* hidden, const float* sgate, void* gx, float* gw1, float* gw2, int B, int HW,
                     int C, int Cr, void* ws, long long ws_bytes, int g16, hyres_stream_t s);
/* ... with the producing PReLU's backward folded in under AMP (round 6): pre fp16 (fp16 activations); g16 = 1: gy /
 * gx fp16 (the gradient rounded to fp16 before the PReLU, as the unfused chain stores it). As hyres_se_bwd_prelu. */
int hyres_se_bwd_prelu_f16(const void* x, const void* gy, const float* w1, const float* w2, const float* pooled,
                           const float* hidden, const float* sgate, void* gx, float* gw1, float* gw2, int B, int HW, int C,
                           int Cr, const void* pre, const float* slope, float* dslope, void* ws, long long ws_bytes,
                           int g16, hyres_stream_t s);
int hyres_spatial_attn_bwd_f16(const void* x, const float* w, const float* pooled2, const int* argmax,
                               const float* attn, const void* gy, void* gx, float* gw, int B, int H, int W,
                               int C, void* ws, long long ws_bytes, int g16, hyres_stream_t s);
/* bilinear backward over fp16 gy / gx (AMP fp16 gradients; fp32 sums; 8B-aligned when C % 4 == 0) */
int hyres_bilinear_bwd_f16(const void* gy, int ldgy, void* gx, int ldgx, int B, int Hi, int Wi, int Ho, int Wo,
                           int C, float scale_h, float scale_w, int accumulate, hyres_stream_t s);
/* Round 6: the up-sample's backward with the PReLU backward of the layer that produced its input folded in
 * (MultiScaleRefine scales 2 / 3: conv + PReLU, then the bilinear up-sample, enhancement.py:89-103): writes
 * gx = pre > 0 ? g : slope * g (g = the gather sum, rounded to fp16 first with fp16 gradients) — NOT accumulated, the
 * caller is the first writer — and ADDS dslope += sum_{pre <= 0} pre * g (deterministic block partials in ws).
 * io: bit 0 gy / gx fp16, bit 1 pre fp16. C % 4 == 0, aligned rows; ws >= hyres_bilinear_bwd_prelu_workspace_bytes. */
long long hyres_bilinear_bwd_prelu_workspace_bytes(int B, int Hi, int Wi, int C);
int hyres_bilinear_bwd_prelu(const void* gy, int ldgy, void* gx, int ldgx, int B, int Hi, int Wi, int Ho, int Wo, int C,
                             float scale_h, float scale_w, const void* pre, int ldpre, const float* slope, float* dslope,
                             void* ws, long long ws_bytes, int io, hyres_stream_t s);

/* ------------------------------------------------------------------------------------------ */
/* losses and optimiser (src/losses/rd_loss.py:18-44, src/utils/engine.py:56-90)              */
/* ------------------------------------------------------------------------------------------ */
/* out[0] (+)= sum(log(x)) over n floats (two-pass deterministic) */
int hyres_sum_log(const float* x, long long n, float* out, void* ws, long long ws_bytes,
                  hyres_stream_t s);
/* out[0] = sum((a-b)^2) */
int hyres_sum_sqdiff(const float* a, const float* b, long long n, float* out, void* ws,
                     long long ws_bytes, hyres_stream_t s);
long long hyres_reduce_workspace_bytes(long long n);
/* g = coef / x  (d/dx of coef*log x) ; g = coef*(a-b) */
int hyres_scale_recip(const float* x, const float* coef, float scale, float* g, long long n,
                      hyres_stream_t s);
int hyres_scale_diff(const float* a, const float* b, const float* coef, float scale, float* g,
                     long long n, hyres_stream_t s);
/* RateDistortionLoss scalars from sums = [sum log lik_y, sum log lik_z, sum sq err]:
 * *out[i] = [loss, bpp, residual_bpp, y_bpp, z_bpp, mse][i]  (rd_loss.py:23-42, alpha = 0) */
int hyres_rd_finalize(const float* sums, const float* jpeg_bpp, float lmbda, long long npx,
                      long long nel, float* const* out, hyres_stream_t s);
/* backward coefficients from the six output gradients: coef = [c_y, c_z, c_mse] */
int hyres_rd_bwd_coef(const float* g0, const float* g1, const float* g2, const float* g3,
                      const float* g4, const float* g5, float lmbda, long long npx, long long nel,
                      float* coef, hyres_stream_t s);
/* sum of squares of a flat buffer, accumulated and returned in fp64 -> out[0] (device double): a finite
 * gradient never overflows it, so !isfinite(out[0]) <=> some element is inf/NaN (GradScaler found_inf is
 * element-wise, torch/amp/grad_scaler.py) and the clip norm of engine.py:76 stays exact; ws >= 8 bytes per
 * block (hyres_reduce_workspace_bytes). */
int hyres_sumsq(const float* x, long long n, double* out, void* ws, long long ws_bytes, hyres_stream_t s);
/* fused Adam over a flat parameter buffer: torch.optim.Adam (foreach, amsgrad=False, weight_decay=0)
 * replacing src/utils/engine.py:68-82 (clip_grad_norm_ -> [GradScaler] -> Adam.step). Hyper-parameters
 * are doubles: 1-beta, the bias corrections, step_size and sqrt(bc2) are formed in double precision as
 * torch does in Python, then used as fp32 scalars. step_dev: device float = completed steps (incremented
 * on device unless the step is skipped). sumsq (device, may be NULL): sum of squares of ``grad``;
 * with max_norm > 0 the clip_grad_norm_ factor min(1, max_norm/(||g*gscale||+1e-6)) is applied on the
 * fly. gscale (device, may be NULL): GradScaler unscale factor 1/scale. skip: 0 never, 1 skip when
 * sumsq is not finite (GradScaler.step's found_inf), 2 skip when sumsq is NaN (engine.py:60-74). */
int hyres_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, long long n,
                    double lr, double beta1, double beta2, double eps, float* step_dev,
                    const double* sumsq, double max_norm, const float* gscale, int skip,
                    hyres_stream_t s);
/* torch GradScaler.update on the device (engine.py:73,80): found_inf = !isfinite(sumsq[0]) of the
 * scaled gradients; scale *= backoff on inf, *= growth after growth_interval clean steps;
 * inv_scale = 1/scale. */
int hyres_grad_scaler_update(const double* sumsq, float* scale, float* inv_scale, int* growth_tracker,
                             double growth_factor, double backoff_factor, int growth_interval,
                             hyres_stream_t s);

/* ------------------------------------------------------------------------------------------ */
/* VGG16 perceptual loss (src/losses/vgg16.py, rd_loss.py:40), NHWC           */
/* ------------------------------------------------------------------------------------------ */
/* torchvision Normalize: y = (x - mean[c]) / std[c], C <= 4; mean / stdv are HOST arrays
 * (vgg16.py:35-38, 50-51) */
int hyres_normalize_fwd(const float* x, float* y, long long P, int C, const float* mean, const float* stdv,
                        hyres_stream_t s);
int hyres_normalize_bwd(const float* g, float* gx, long long P, int C, const float* mean, const float* stdv,
                        int accumulate, hyres_stream_t s);
/* y = max(x, 0) (nn.ReLU at a slice boundary, vgg16.py:29-33) */
int hyres_relu_fwd(const float* x, float* y, long long n, hyres_stream_t s);
/* nn.MaxPool2d(2, 2): argmax in {0..3} ((0,0),(0,1),(1,0),(1,1)), first maximum wins, NaN propagates */
int hyres_maxpool2_fwd(const float* x, float* y, unsigned char* argmax, int B, int H, int W, int C, hyres_stream_t s);
int hyres_maxpool2_bwd(const float* g, const unsigned char* argmax, float* gx, int B, int H, int W, int C,
                       int accumulate, hyres_stream_t s);
/* out[0] (+)= mean |a - b| (two-pass deterministic), its backward ga (+)= coef[0] * sign(a - b) / n
 * (vgg16.py:58 torch.abs(x - y).mean()) */
long long hyres_absdiff_workspace_bytes(long long n);
int hyres_absdiff_mean(const float* a, const float* b, long long n, float* out, int accumulate, void* ws,
                       long long ws_bytes, hyres_stream_t s);
int hyres_absdiff_bwd(const float* a, const float* b, const float* coef, long long n, float* ga, int accumulate,
                      hyres_stream_t s);

/* ------------------------------------------------------------------------------------------ */
/* entropy coding (compress / decompress): compressai 1.2.6 semantics            */
/* ------------------------------------------------------------------------------------------ */
/* GaussianConditional.build_indexes(scales) + quantize(y, "symbols", means) of one checkerboard pass
 * (models/checkerboard.py:159-161): params NHWC [B,H,W,ldp] with scales in channels [0,M) and means in
 * [M,2M); y NHWC masked by parity (0 anchor, 1 non-anchor, -1 none); sym/idx int32 NCHW. y == NULL:
 * indexes only (decoder side). */
int hyres_gc_symbols(const float* y, int ldy, const float* params, int ldp, int M, int B, int H, int W, int parity,
                     const float* scale_table, int nt, int* sym, int* idx, hyres_stream_t s);
/* GaussianConditional.decompress's dequantize: out[NHWC] (+)= sym + means (checkerboard.py:162-164) */
int hyres_gc_dequant(const int* sym, const float* params, int ldp, int M, int B, int H, int W, float* out, int ldo,
                     int accumulate, hyres_stream_t s);
/* EntropyBottleneck.compress/decompress symbolisation around the channel medians (checkerboard.py:170-171):
 * dequant = 0: sym = round(z - med); 1: zhat = sym + med */
int hyres_eb_symbols(const float* z, int ldz, const float* medians, int B, int H, int W, int C, int* sym,
                     float* zhat, int ldo, int dequant, hyres_stream_t s);
/* compressai pmf_to_quantized_cdf (cpp_exts/ops/ops.cpp): n probabilities -> n+1 CDF entries summing to
 * 2^precision with every symbol frequency >= 1 (host) */
int hyres_pmf_to_quantized_cdf(const float* pmf, int n, int precision, int* cdf_out);
/* compressai RansEncoder.encode_with_indexes / RansDecoder.decode_with_indexes (cpp_exts/rans): 64-bit
 * rANS, 16-bit CDFs [ncdf][cdf_stride], bypass escape for out-of-range symbols (host). out == NULL:
 * *out_len = the string length only. */
int hyres_rans_encode_with_indexes(const int* symbols, const int* indexes, long long n, const int* cdfs,
                                   int cdf_stride, const int* cdf_sizes, const int* offsets, int ncdf,
                                   unsigned char* out, long long out_cap, long long* out_len);
int hyres_rans_decode_with_indexes(const unsigned char* in, long long in_len, const int* indexes, long long n,
                                   const int* cdfs, int cdf_stride, const int* cdf_sizes, const int* offsets,
                                   int ncdf, int* symbols_out);

#ifdef __cplusplus
}
#endif
#endif /* HYRES_HIP_H */
