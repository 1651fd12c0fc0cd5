// Host-callable launchers of the ldnn gfx950 kernels (no torch dependency:
// every launcher takes raw device pointers and a hipStream_t, so the same
// entry points serve the pybind layer, graph capture and C++ tests).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ldnn {

enum Epilogue : int {
  EPI_NONE = 0,
  EPI_BIAS = 1,
  EPI_BIAS_RELU = 2,
  EPI_BIAS_SIGMOID = 3,
  EPI_DRELU = 4,
  EPI_DSIGMOID = 5,
  // fp32-output weight-gradient GEMMs only: the epilogue applies the optimizer to
  // the weights instead of storing the gradient (GemmParams::opt)
  EPI_OPT_SGD = 6,
  EPI_OPT_ADAM = 7,
  // four-wave kernel (gemm_q.hip) only: ReLU as a bit mask instead of the bf16
  // activation -- the forward writes mask_out[m][n/8] (bit q = output (m, n+q) > 0)
  // beside the activation; the dgrad reads mask_in instead of 16 B of aux per 8 columns
  EPI_BIAS_RELU_MASK = 8,
  EPI_DRELU_MASK = 9,
  // four-wave kernel only, bf16 out, no split-K: bias + ReLU forward of the last hidden
  // layer that also multiplies its output tile by the classifier head's weight
  // (head_w, <= 16 classes) on the MFMA pipe: head_part[n0 / 256][m][0..15] = the
  // tile's partial logits (summed by head_xent_parts)
  EPI_BIAS_RELU_HEAD = 10,
};

// Fused optimizer epilogue: gradient element (m, n) updates master[m*ldc + n].
struct OptEpi {
  float* master;          // fp32 weights (ldc row stride, like C)
  float* m;               // SGD momentum / Adam exp_avg (nullable for momentum-free SGD)
  float* v;               // Adam exp_avg_sq
  uint16_t* shadow;       // bf16 copy the GEMMs read (nullable)
  const float* hp;        // device [lr, step]
  float grad_scale, momentum, dampening, weight_decay, beta1, beta2, eps;
  int nesterov, decoupled;
};

struct GemmParams {
  const uint16_t* A;
  const uint16_t* B;
  void* C;
  const float* bias;     // [N] fp32 (EPI_BIAS*)
  const uint16_t* aux;   // [M][ldaux] bf16 saved activation (EPI_D*)
  float* dbias;          // optional [N] fp32 column-sum accumulator
  int M, N, K;
  int lda, ldb, ldc, ldaux;
  float beta;            // fp32 output only: C = acc + beta * C
  int splitk;            // >1: K split over gridDim.y (128-tile): fp32 atomics into C (EPI_NONE, fp32 out)
                         //     or, with ws/cnt, an in-launch deterministic combine (any epilogue)
  int direct_epi;        // 256-tile bf16 outputs: 1 = per-fragment stores (A/B knob), 0 = LDS-staged rows
  int variant;           // 256-tile main loop: 0/1 = 2-stage BK64 (default), 2 = 4-slot BK32 ring, 3 = 5-slot ring
  float* ws;             // split-K combine: [tiles][splitk] slabs of 64 KiB (gemm_splitk_ws_bytes)
  int* cnt;              // split-K combine: [tiles] arrival counters, zero before the first launch
  OptEpi opt;            // EPI_OPT_*: the weights this gradient updates
  int64_t c_split_stride;  // gemm_q split-K (gridDim.y > 1) without a combine: split y writes its
                           // partial product to C + y * c_split_stride elements (then slab_sum)
  uint8_t* mask_out;       // EPI_BIAS_RELU_MASK: [M][ldmask] ReLU bits
  const uint8_t* mask_in;  // EPI_DRELU_MASK: [M][ldmask] ReLU bits of the saved activation
  int ldmask;              // bytes per mask row (>= N / 8)
  const uint16_t* head_w;  // EPI_BIAS_RELU_HEAD: [16][ldhw] bf16 head weight (rows >= classes zero)
  float* head_part;        // EPI_BIAS_RELU_HEAD: [ceil(N / 256)][M][16] fp32 partial logits
  int ldhw;
};
// Workspace of the in-launch split-K combine of a 128-tile GEMM (bytes; counters = tiles).
size_t gemm_splitk_ws_bytes(int M, int N, int splitk);
int gemm_tiles128(int M, int N);

// Picks the tiling (256x256 LDS-DMA kernel or 128x128 kernel) from the shape.
hipError_t gemm_bf16(const GemmParams& p, bool a_kcontig, bool b_kcontig, int epi, bool out_f32,
                     hipStream_t s);
// Same with an explicit tile (128 or 256); 256 falls back to 128 for operands >= 2 GiB.
hipError_t gemm_bf16_tile(const GemmParams& p, bool a_kcontig, bool b_kcontig, int epi, bool out_f32, int tile,
                          hipStream_t s);
int gemm_pick_tile(int M, int N, int K, bool out_f32);
// Four-wave 256x256 kernel (gemm_q.hip, 128x128 per wave): same contract as
// gemm_bf16; p.splitk > 1 needs the in-launch combine workspace p.ws
// (gemm_q_ws_bytes) and p.cnt (gemm_q_tiles zeroed counters).  Operands must each
// be < 2 GiB.
hipError_t gemm_q(const GemmParams& p, bool a_kcontig, bool b_kcontig, int epi, bool out_f32, hipStream_t s);
size_t gemm_q_ws_bytes(int M, int N, int splitk);
int gemm_q_tiles(int M, int N);
// Whether gemm_q beats gemm.hip's k256 on a 256-tile shape (measured on MI355X,
// profiles/gemm_q_r2.txt: it loses at short K, where its one-wave-per-SIMD
// prologue/epilogue is not amortised).
inline bool gemm_q_preferred(int M, int N, int K) { return K >= 1024; }
// Split-K factor the 128-tile kernel uses for an fp32 EPI_NONE output (1 = none).
int gemm_pick_splitk(int M, int N, int K);
// Skinny-N forward GEMM (N <= 64, both operands k-contiguous, bf16 out): one
// 16-row strip per workgroup, K split over its 4 waves, reduced in LDS.
hipError_t gemm_skinny_n(const GemmParams& p, int epi, hipStream_t s);
constexpr size_t kOOBLimit = 0x80000000ull;

// ---- implicit-GEMM convolution (conv.hip): NHWC activations, KRSC weights, C/K % 8 == 0
struct ConvShape {
  int N, H, W, C;   // input (C padded to a multiple of 8)
  int K, R, S;      // output channels (padded to a multiple of 8), filter
  int P, Q;         // output spatial size
  int stride, pad;
  int c_real;       // channels of C that carry data (the rest are zero padding); 0 = all C
  int s2d_packed;   // conv2d_fwd with s2d_xs: the image is already packed (nchw_to_nhwc's s2d output)
};
// ws / cnt: optional in-launch split-K workspace for small-M shapes (conv2d_lds_workspace);
// without it those shapes run unsplit.
struct BnFin;  // (BatchNorm finalize state, below)
// bn (optional): also accumulate the following training-mode BatchNorm's statistics
// over the bf16 outputs and finalize them; *bn_done reports whether that happened
// (only the LDS-DMA path does it, for EPI_NONE).
hipError_t conv2d_fwd(const ConvShape& s, const uint16_t* x, const uint16_t* w, uint16_t* y, const float* bias,
                      int epi, hipStream_t st, float* ws = nullptr, int* cnt = nullptr, const BnFin* bn = nullptr,
                      bool* bn_done = nullptr, uint16_t* s2d_xs = nullptr);
// s2d_xs (ResNet-type 7x7 / 2 stems, stem_s2d_fwd_ok): [N][P+3][Q+3][16] buffer the forward packs the
// space-to-depth image into and runs on (conv_s2d_ws_kernel); the weight gradient reuses it
bool stem_s2d_fwd_ok(const ConvShape& s);
struct BnBwdFuse;  // (a BatchNorm backward whose statistics a dgrad epilogue takes, below)
// bnb (optional): dx is the gradient of a training BatchNorm(+ReLU)'s output; also accumulate
// that BN's backward statistics over the bf16 dx and finalize them (*bn_done: whether it did)
hipError_t conv2d_dgrad(const ConvShape& s, const uint16_t* dy, const uint16_t* w, uint16_t* dx, hipStream_t st,
                        float* ws = nullptr, int* cnt = nullptr, const BnBwdFuse* bnb = nullptr,
                        bool* bn_done = nullptr);
hipError_t conv2d_wgrad(const ConvShape& s, const uint16_t* dy, const uint16_t* x, float* dw, float beta,
                        hipStream_t st, float* ws = nullptr, const uint16_t* s2d_xs = nullptr);
// A layer's dgrad (shape sd, as conv2d_dgrad) and wgrad (shape sw, as conv2d_wgrad), both reading
// dy: ONE launch when both take the 4-wave gather kernels (conv2d_bwd_lds), else one by one.
hipError_t conv2d_bwd(const ConvShape& sd, const uint16_t* dy, const uint16_t* w, uint16_t* dx, float* ws_d,
                      int* cnt_d, const BnBwdFuse* bnb, bool* bn_done, const ConvShape& sw, const uint16_t* x,
                      float* dw, float beta, float* ws_w, hipStream_t st);
// LDS-DMA fast path (conv_lds.hip): hipErrorNotSupported outside its shape set
// (fwd needs C % 64 == 0, dgrad K % 64 == 0, stride 1 or 2).
// bn_used: whether the epilogue accumulated the BN statistics (a slab split-K shape does not)
hipError_t conv2d_fwd_lds(const ConvShape& s, const uint16_t* x, const uint16_t* w, uint16_t* y, const float* bias,
                          int epi, hipStream_t st, float* ws, int* cnt, const BnFin* bn = nullptr,
                          bool* bn_used = nullptr, uint16_t* s2d_xs = nullptr);
hipError_t conv2d_dgrad_lds(const ConvShape& s, const uint16_t* dy, const uint16_t* w, uint16_t* dx, hipStream_t st,
                            float* ws, int* cnt, const BnBwdFuse* bnb = nullptr, bool* bn_used = nullptr);
hipError_t conv2d_wgrad_lds(const ConvShape& s, const uint16_t* dy, const uint16_t* x, float* dw, float beta,
                            hipStream_t st, float* ws, const uint16_t* s2d_xs = nullptr);
// A downsampling block's 3x3 conv (s0, w0 -> y0) and 1x1 shortcut conv (s1, w1 -> y1) of one
// input x, each with its optional next-BN statistics: one launch where the kernels allow
// (conv2d_fwd2_lds), else one by one (conv2d_fwd2).
hipError_t conv2d_fwd2(const ConvShape& s0, const uint16_t* x, const uint16_t* w0, uint16_t* y0, float* ws0,
                       int* cnt0, const BnFin* bn0, bool* done0, const ConvShape& s1, const uint16_t* w1,
                       uint16_t* y1, float* ws1, int* cnt1, const BnFin* bn1, bool* done1, hipStream_t st);
hipError_t conv2d_fwd2_lds(const ConvShape& s0, const uint16_t* x, const uint16_t* w0, uint16_t* y0, float* ws0,
                           int* cnt0, const BnFin* bn0, bool* used0, const ConvShape& s1, const uint16_t* w1,
                           uint16_t* y1, float* ws1, int* cnt1, const BnFin* bn1, bool* used1, hipStream_t st);
// One conv's backward job: dgrad (shape sd: dy, w -> dx; split-K workspace ws_d / counters
// cnt_d) and wgrad (shape sw: dy, x -> dw with beta; slabs ws_w).
struct BwdJob {
  ConvShape sd, sw;
  const uint16_t* dy;
  const uint16_t* w;
  uint16_t* dx;
  float* ws_d;
  int* cnt_d;
  float* dw;
  float beta;
  float* ws_w;
};
// A downsampling block's two convs of one input x: both dgrads and wgrads in one launch where the
// kernels allow (conv2d_bwd2_lds), else each conv's conv2d_bwd (conv2d_bwd2).  j0 / j1 need
// distinct counter ranges.
hipError_t conv2d_bwd2(const BwdJob& j0, const BwdJob& j1, const uint16_t* x, hipStream_t st);
hipError_t conv2d_bwd2_lds(const BwdJob& j0, const BwdJob& j1, const uint16_t* x, hipStream_t st);
// hipErrorNotSupported: the pair does not share a launch (conv2d_bwd runs them one by one)
hipError_t conv2d_bwd_lds(const ConvShape& sd, const uint16_t* dy, const uint16_t* w, uint16_t* dx, float* ws_d,
                          int* cnt_d, const BnBwdFuse* bnb, bool* bn_used, const ConvShape& sw, const uint16_t* x,
                          float* dw, float beta, float* ws_w, hipStream_t st);
// dgrad + wgrad in one launch (LDNN_CONV_PAIR: 0 off, 1 / 3 (default) / 2 see conv_lds.hip;
// the setter is for tests / A/B)
void set_conv_pair(int on);
int get_conv_pair();
struct ConvWorkspace {
  size_t slab_bytes = 0;  // fp32 split-K slabs (0: the shape runs unsplit)
  int counters = 0;       // int arrival counters, zeroed
};
// op 0 = fwd, 1 = dgrad (in-launch combine: slabs + counters), 2 = wgrad (partial slabs, no counters)
ConvWorkspace conv2d_lds_workspace(const ConvShape& s, int op);
// 0 = LDS-DMA fast path where it applies (default), 1 = generic kernel only (A/B and tests)
void set_conv_impl(int impl);
int get_conv_impl();
// halo-staged 3x3 stride-1 conv path (conv_lds.hip): 0 = off, 1 = default dispatch
// (dgrad + 256x64 fwd tiles), 2 = also the 128x128 fwd tiles
void set_conv_stem_s2d(int mode);   // 0: split-K stem wgrad, 1: space-to-depth stem wgrad (default)
void set_conv_wgrad_ring(int mode);  // 0: split-K wgrad everywhere, 1: the ring wgrad for 3x3 stride-1 convs
void set_conv_halo(int mode);
void set_conv_hb(int mode);
int get_conv_hb();
// weight-stationary 64 -> 64 channel 3x3 conv: 0 off, 1 on (default)
void set_conv_ws(int mode);  // see conv_lds.hip ws_env
int get_conv_ws();
// phase-trace buffer ([workgroup][4] uint64) of the LDNN_CONV_XF=32 diagnostic build (nullptr: off)
// in-launch split-K combine of the LDS-DMA convs: 1 = the tile's last K slice sums, 0 = the last arrival
void set_conv_combine_last(int on);
int get_conv_combine_last();
// dgrad-side BN backward statistics: 0 off, 1 slab split-K sum only, 2 also the direct / combine
// epilogue (LDNN_CONV_BN_BWD; the setter is for tests)
void set_conv_bn_bwd(int mode);
int get_conv_bn_bwd();
void set_conv_trace(uint64_t* buf);
int get_conv_halo();

// ---- BatchNorm / pooling on NHWC bf16 (bn_pool.hip), C % 8 == 0
struct BnArgs {
  const uint16_t* x;          // [M][C] input
  const uint16_t* residual;   // optional [M][C] added before the ReLU
  uint16_t* y;                // [M][C] output (also read by backward when relu)
  const float* gamma;         // [C] (nullable: affine=False)
  const float* beta;
  float* running_mean;        // [C] (nullable: no EMA / eval uses them)
  float* running_var;
  float* save_mean;           // [C] batch statistics kept for backward
  float* save_invstd;
  float* scale;               // unused (kept for layout compatibility): scale / shift live in ws
  float* shift;
  float* ws;                  // [bn_workspace_floats(C)] fp32, zeroed ONCE by the owner and kept
                              // (accumulators are cleared by the kernels that consume them)
  int M, C;
  float eps, momentum;
  int training, relu;
  int64_t* num_batches;       // optional BatchNorm2d.num_batches_tracked, += 1 per training forward
  uint8_t* mask;              // optional [M][C/8] ReLU bits: written by a relu forward, read by the
                              // backward instead of y (1/16 of y's bytes per read)
  const uint16_t* dy2;        // backward: optional second gradient of y, summed with dy on the fly
                              // (a residual block's shortcut-branch gradient: no separate add pass)
};
int bn_workspace_floats(int C);
hipError_t bn_forward(const BnArgs& a, hipStream_t s);
struct BnFin {
  float* acc;                 // [2C] accumulators (left zeroed for the next call)
  int* ticket;                // arrival counter (left zero)
  const float* gamma;
  const float* beta;
  float* running_mean;
  float* running_var;
  float* save_mean;           // fwd: written; bwd: read
  float* save_invstd;
  float* coef;                // fwd: scale | shift ; bwd: A | B | D
  float* dgamma;              // bwd: accumulated (grad_assign: overwritten)
  float* dbeta;
  int grad_assign;            // bwd: 1 = dgamma / dbeta = the totals (first write of the step)
  int64_t* num_batches;       // fwd: += 1 (BatchNorm2d.num_batches_tracked), nullable
  float eps, momentum;
  float* part;                // [kGrpMax][2C] row-group partials of the grouped reduce (ldnn_bn_fin.h)
  int* tickets;               // its per-64-channel-column tickets (left zero)
};
// The backward statistics of a BN(+ReLU) taken by the epilogue of the dgrad that produces the
// gradient of its output: sum g and sum g * (x - mean) * invstd, g = dy * relu'(y) (mask bits)
struct BnBwdFuse {
  BnFin fin;                  // bn_backward_fin_conv: the BN's backward finalize state
  const uint16_t* x;          // [M][C] the BN's input
  const uint8_t* mask;        // [M][C/8] its ReLU bits (nullptr: no ReLU)
};
// Training-mode forward finalize state of a BN (its ws accumulators / ticket / coef).
BnFin bn_forward_fin(const BnArgs& a);
// ... for a producing conv's epilogue (its kBnCopies accumulator copies in ws).
BnFin bn_forward_fin_conv(const BnArgs& a);
// The apply pass alone, with the scale / shift a fused statistics pass left in a.ws.
hipError_t bn_forward_apply(const BnArgs& a, hipStream_t s);
// dx (and optionally dres = upstream gradient after the ReLU mask, for the residual
// branch); dgamma / dbeta are ACCUMULATED (flat gradient buffer)
// stats_ready: a dgrad epilogue already finalized the backward coefficients into a.ws
// (conv2d_dgrad with a BnBwdFuse): the apply pass alone
hipError_t bn_backward(const BnArgs& a, const uint16_t* dy, uint16_t* dx, uint16_t* dres, float* dgamma,
                       float* dbeta, hipStream_t s, bool grad_assign = false, bool stats_ready = false);
// Backward finalize state of a BN for a producing dgrad's epilogue (its ws accumulators / coef).
BnFin bn_backward_fin_conv(const BnArgs& a, float* dgamma, float* dbeta, bool grad_assign);
// Residual block tail with a BatchNorm on both branches: y = relu(bn_a(a.x) + bn_b(b.x)), the
// shortcut BN's output never stored (a.relu, both training mode; ready_*: statistics already
// finalized into the ws by the producing convs).  a.y / a.mask: the output and its ReLU bits.
hipError_t bn_dual_forward(const BnArgs& a, const BnArgs& b, bool ready_a, bool ready_b, hipStream_t s);
// its backward: dx = d/d a.x, dr = d/d b.x from dy (+ a.dy2); dgamma / dbeta as bn_backward
hipError_t bn_dual_backward(const BnArgs& a, const BnArgs& b, const uint16_t* dy, uint16_t* dx, uint16_t* dr,
                            float* dgamma_a, float* dbeta_a, float* dgamma_b, float* dbeta_b, bool assign_a,
                            bool assign_b, hipStream_t s);
// relu(BN(x)) -> 3x3/2 max-pool in one pass (a.x = [N][H][W][C] pre-BN, a.M = N*H*W, a.relu = 1):
// y [N][P][Q][C] pooled, arg [N][P][Q][C] window argmax (0xff: the max was clamped by the ReLU).
// stats_ready: scale / shift already in a.ws (the producing conv's epilogue finalized them).
// Needs C / 8 to divide 256.
hipError_t bn_maxpool_forward(const BnArgs& a, int N, int H, int W, int P, int Q, int pad, uint16_t* y,
                              uint8_t* arg, bool stats_ready, hipStream_t s, uint16_t* xam = nullptr);
// (xam: optional [N][P][Q][C] output, the BN input at each argmax -- what the backward statistics read)
// its backward: dx [N][H][W][C] from the pooled gradient dy (+ a.dy2), dgamma / dbeta as bn_backward;
// with the forward's xam the statistics pass reads the pooled-size xam / dy / argmax instead of x
hipError_t bn_maxpool_backward(const BnArgs& a, int N, int H, int W, int P, int Q, int pad, const uint16_t* dy,
                               const uint8_t* arg, uint16_t* dx, float* dgamma, float* dbeta, hipStream_t s,
                               bool grad_assign = false, const uint16_t* xam = nullptr);
hipError_t pool2d_fwd(const uint16_t* x, uint16_t* y, uint8_t* argmax, int N, int H, int W, int C, int P, int Q,
                      int R, int S, int stride, int pad, bool is_max, hipStream_t s, int nchw_c = 0);
// nchw_c > 0: y (fwd) / dy (bwd) is a dense NCHW tensor of the first nchw_c channels (argmax stays NHWC)
hipError_t pool2d_bwd(const uint16_t* dy, const uint8_t* argmax, uint16_t* dx, int N, int H, int W, int C, int P,
                      int Q, int R, int S, int stride, int pad, bool is_max, hipStream_t s,
                      const uint16_t* dy2 = nullptr, int nchw_c = 0);
hipError_t global_avgpool_fwd(const uint16_t* x, uint16_t* y, int N, int HW, int C, hipStream_t s);
hipError_t global_avgpool_bwd(const uint16_t* dy, uint16_t* dx, int N, int HW, int C, hipStream_t s);

// ---- elementwise / activations (bf16 storage, fp32 math) ---------------------
enum Act : int { ACT_RELU = 0, ACT_SIGMOID = 1 };
hipError_t act_fwd(const uint16_t* x, uint16_t* y, int64_t n, int act, hipStream_t s);
hipError_t act_bwd(const uint16_t* dy, const uint16_t* y, uint16_t* dx, int64_t n, int act, hipStream_t s);
// dbias[c] (+)= sum_r x[r][c] over a [rows][cols] bf16 matrix (ld = cols).  ws (optional): a zeroed
// scratch of cols floats + one int the caller keeps; an overwriting sum over several row groups then
// runs as ONE launch (ticketed: the last group moves the sums into out and re-zeroes ws)
hipError_t colsum_bf16(const uint16_t* x, float* out, int rows, int cols, bool accumulate, hipStream_t s,
                       float* ws = nullptr);
// dx = act'(y) * dy with the column sums of dx added to out (dy may alias dx); ws as colsum_bf16
hipError_t act_bwd_colsum(const uint16_t* dy, const uint16_t* y, uint16_t* dx, float* out, int rows, int cols,
                          int act, bool accumulate, hipStream_t s, float* ws = nullptr);
hipError_t cast_f32_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t s);
// graph-capture-safe zero fill of a strided fp32 block (instead of hipMemset2DAsync)
hipError_t zero2d_f32(float* p, int rows, int cols, int ld, hipStream_t s);
// out[c][r] = in[r][c], bf16, rows / cols / strides multiples of 8
hipError_t transpose_bf16(const uint16_t* in, uint16_t* out, int rows, int cols, int ldi, int ldo, hipStream_t s);
// NCHW (fp32 / bf16) -> NHWC bf16 [N][HW][cp], pad channels zeroed (cp % 8 == 0)
hipError_t nchw_to_nhwc(const void* src, bool src_f32, uint16_t* dst, int N, int C, int HW, int cp, hipStream_t s,
                        const void* extra_src = nullptr, void* extra_dst = nullptr, int64_t extra_bytes = 0);
// The same for a <= 4-channel input of even H, W into an 8-channel dst, also writing the stem's 2x2
// space-to-depth image s2d[N][H/2+3][W/2+3][16] (conv_stem.hip stem_s2d_pack_kernel's layout) in the pass.
hipError_t nchw_to_nhwc_s2d(const void* src, bool src_f32, uint16_t* dst, uint16_t* s2d, int N, int C, int H,
                            int W, hipStream_t s, const void* extra_src, void* extra_dst, int64_t extra_bytes);
// sum split-K slabs [splits][rows][ldw] into out[rows][ncols] (stride ldo); extra[r] = column ncols
hipError_t slab_sum_cols(const float* ws, int splits, int rows, int ldw, float* out, int ldo, int ncols, float* extra,
                         hipStream_t s);
hipError_t cast_bf16_f32(const uint16_t* x, float* y, int64_t n, hipStream_t s);
// y = a*x + b*y1 + c*y2 (fp32, in place on x allowed); optional bf16 shadow of y
hipError_t mix3_f32(float* out, const float* x, const float* y1, const float* y2, float a, float b, float c,
                    int64_t n, uint16_t* shadow, hipStream_t s);
// mix3_f32 with bf16 y1 / y2 (the bf16 copies a per-step gossip exchange receives)
hipError_t mix3_y16(float* out, const float* x, const uint16_t* y1, const uint16_t* y2, float a, float b, float c,
                    int64_t n, uint16_t* shadow, hipStream_t s);
// x *= scale (fp32), optional bf16 shadow
hipError_t scale_f32(float* x, float scale, int64_t n, uint16_t* shadow, hipStream_t s);

// ---- fused softmax cross-entropy (K14 + K15 of SURVEY §2.3) ---------------
// logits [B][ld] bf16 (first C columns valid), labels int64 [B].
// Writes dlogits [B][ld] bf16 = (softmax - onehot) * grad_scale (padded columns 0),
// accumulates sum of per-row loss into stats[0] and #correct into stats[1]
// (fp32), optionally column sums of dlogits into dbias[ld].
// With fin.out set the per-row sums go to fin.acc (2 floats + an arrival counter,
// zero at entry and left zero: a persistent workspace) and the last block writes
// fin.out = [loss_sum * fin.scale, #correct], adds both into `stats` if given --
// the loss scalar and the running statistics with no fill / divide / add launches.
struct XentFin {
  float* out = nullptr;
  float* acc = nullptr;
  unsigned* cnt = nullptr;
  float scale = 1.f;
};
hipError_t softmax_xent(const uint16_t* logits, const int64_t* labels, uint16_t* dlogits, float* stats,
                        float* dbias, int B, int C, int ld, float grad_scale, hipStream_t s,
                        const XentFin* fin = nullptr);
// out[i] = src[i] * (*scale) over n bf16 (the loss backward's grad_output, read on the device)
hipError_t scale_bf16_dev(const uint16_t* src, const float* scale, uint16_t* out, int64_t n, hipStream_t s);
// overlap-probe communication stand-in: `reps` copies of src on `blocks` workgroups
hipError_t standin_copy(const float* src, float* dst, int64_t n, int blocks, int reps, hipStream_t s);

// ---- pooled classifier head (gap_head.hip): global average pool + Linear (<= 16 classes)
bool gap_linear_ok(int N, int HW, int C, int ncls);
hipError_t gap_linear_fwd(const uint16_t* x, const uint16_t* W, const float* b, uint16_t* pooled, uint16_t* logits,
                          int N, int HW, int C, int ldw, int ncls, int ldl, hipStream_t s);
hipError_t gap_linear_bwd(const uint16_t* g, const uint16_t* pooled, const uint16_t* W, float* dW, float* db,
                          uint16_t* dx, int N, int HW, int C, int ldg, int ldw, int lddw, int ncls, float beta_w,
                          float beta_b, hipStream_t s);

// ---- fused optimizers over flat fp32 buffers -------------------------------
// hp (device fp32): [0]=lr [1]=step (already incremented for Adam) ; grad_scale multiplies g
// Gradient ranges [zb[i], ze[i]) (element offsets into this launch's range) are
// zeroed after being consumed: accumulate-into (atomic) gradient producers of the
// next step then need no separate zeroing launch.
struct GradZero {
  int64_t zb[2] = {0, 0}, ze[2] = {0, 0};
};
struct SgdParams {
  float momentum, dampening, weight_decay;
  int nesterov;
  int first_step;  // momentum buffer initialised from g (torch semantics)
  GradZero zero;
};
// grid cap of the optimizer kernels launched from now on (0 = default 2048 blocks)
void set_opt_max_blocks(int n);
// one [rows][cols] matrix of the range (at element `begin`) whose bf16 shadow is also written
// transposed into `out` ([cols][rows]); rows, cols multiples of 64
struct ShadowT {
  int64_t begin = 0;
  int rows = 0, cols = 0;
  uint16_t* out = nullptr;
};
hipError_t sgd_step(float* param, float* grad, float* mom, uint16_t* shadow, const float* hp,
                    float grad_scale, SgdParams sp, int64_t n, hipStream_t s, const ShadowT* tr = nullptr);
struct AdamParams {
  float beta1, beta2, eps, weight_decay;
  int decoupled;  // AdamW
  GradZero zero;
};
hipError_t adam_step(float* param, float* grad, float* m, float* v, uint16_t* shadow, const float* hp,
                     float grad_scale, AdamParams ap, int64_t n, hipStream_t s);
// hp[1] += 1 (graph-capturable step counter)
hipError_t bump_step(float* hp, hipStream_t s);

// ---- classifier head (<= 64 classes): fused Linear + softmax-xent, and its wgrad
struct HeadParams {
  const uint16_t* h;      // [B][ldh] bf16 input features
  const uint16_t* W;      // [ldw_rows][ldw] bf16 weight (rows >= C zero-padded)
  const float* bias;      // [ld] fp32 (zero-padded)
  const int64_t* labels;  // [B]
  uint16_t* logits;       // [B][ld] bf16 (optional)
  uint16_t* dlogits;      // [B][ld] bf16, softmax - onehot, times grad_scale
  float* stats;           // [ceil(B/16)][2] per-workgroup (loss sum, correct) accumulators
  int B, K, C, ld, ldh, ldw, ldw_rows;
  float grad_scale;
  // optional fused dgrad of the head (K <= head_dgrad_max_k()):
  // dh = (dlogits W) * act'(h) [B][lddh] bf16, dbias += column sums of dh
  uint16_t* dh;
  float* dbias;         // += column sums of dh (via dbias_ws: head_dgrad_ws_floats(B, K) floats)
  float* dbias_ws;
  int lddh, dgrad_epi;  // EPI_NONE / EPI_DRELU / EPI_DSIGMOID
  // 0: forward-only head kernel + the streaming dgrad kernel (needs ld == 16; dbias by
  //    atomics, no dbias_ws); 1: dgrad fused into the head kernel, h re-read from
  //    global memory; 2: fused, h staged in LDS (1 / 2 need K <= head_dgrad_max_k()
  //    and dbias_ws for dbias)
  int dgrad_mode;
  // head_bwd only: dW [nrows_w][lddw] fp32 += dlogits^T h, db [nrows_w] += column sums of dlogits
  float* dW;
  float* db;
  int lddw, nrows_w;
};
hipError_t head_fwd_xent(const HeadParams& p, hipStream_t s);
// Softmax-xent + argmax of logits = bias + sum_s parts[s][b][0..15] (the partial logits
// of an EPI_BIAS_RELU_HEAD forward, ld == 16): writes logits / dlogits / stats exactly
// like head_fwd_xent (p.h / p.W unused).
hipError_t head_xent_parts(const HeadParams& p, const float* parts, int nparts, hipStream_t s);
// The streaming head dgrad alone (head_fwd_xent's dgrad_mode 0 second launch):
// dh = (dlogits W) * act'(h), dbias += column sums of dh; needs ld == 16.
hipError_t head_dgrad_stream(const HeadParams& p, hipStream_t s);
// The head's dgrad (head_dgrad_stream's outputs) AND wgrad (head_wgrad's, accumulated into a
// pre-cleared dW / db by fp32 atomics) in one pass over h, both products on the MFMA pipe;
// needs ld == 16, K % 64 == 0, dgrad_epi EPI_NONE / EPI_DRELU, dbias (if any) pre-cleared.
hipError_t head_bwd(const HeadParams& p, hipStream_t s);
int head_dgrad_max_k();
size_t head_dgrad_ws_floats(int B, int K);
// out[i] = sum_s ws[s][i] (+ beta * out[i]) over n4 float4 columns and `splits` slabs
hipError_t slab_sum(const float* ws, float* out, int64_t n4, int splits, float beta, hipStream_t s);
struct HeadWgradParams {
  const uint16_t* dz;  // [B][ld] bf16
  const uint16_t* h;   // [B][ldh] bf16
  float* dW;           // [nrows][lddw] fp32
  float* db;           // [nrows] fp32 (optional)
  int B, K, ld, ldh, lddw, nrows;
};
// splits > 1 accumulate with atomics into dW / db, which must be cleared; splits <= 0: auto
hipError_t head_wgrad(const HeadWgradParams& p, int splits, hipStream_t s);
int head_wgrad_splits(int B, int K);

// ---- synthetic data (K20): deterministic device-side generator -----------
hipError_t synth_normal_bf16(uint16_t* x, int64_t n, uint64_t seed, float stddev, hipStream_t s);
hipError_t synth_labels(int64_t* y, int64_t n, int classes, uint64_t seed, hipStream_t s);

// ---- input pipeline (K20): gather + AutoAugment / flip+crop + normalise -----
constexpr int kAugOps = 15, kAugBins = 10, kAugPolicySlots = 64;
struct AugParams {
  const uint8_t* images;  // [n_images][C][H][W] uint8, resident dataset
  const int64_t* index;   // [B] dataset rows of the batch
  void* out;              // [B][C][H][W] bf16 or fp32: x * a[c] + b[c]
  const float* a;         // [C]
  const float* b;         // [C]
  int64_t n_images;
  int B, C, H, W;
  uint64_t seed;          // batch seed (per-sample draws are counter hashes of it)
  int mode;               // bit0 AutoAugment policy, bit1 random flip + padded crop
  int pad;                // crop padding
  int fixed_op, fixed_bin, fixed_sign;  // fixed_op >= 0: apply only this op (tests)
  int n_policies;         // sub-policies (2 slots each)
  float mags[kAugOps][kAugBins];
  float rot_cos[kAugBins], rot_sin[kAugBins];
  int pol_op[kAugPolicySlots];
  float pol_prob[kAugPolicySlots];
  int pol_bin[kAugPolicySlots];
  int signed_op[kAugOps];
};
// largest C*H*W the LDS-resident kernel takes (two ping-pong images + scratch)
constexpr int kAugMaxPixels = 28 * 1024;
hipError_t augment_batch(const AugParams& p, bool out_f32, hipStream_t s);


// ---- one-shot intra-node all-reduce over IPC-mapped peer buffers (ipc.hip) ----
constexpr int kIpcMaxRanks = 8;     // one MI355X node
constexpr int kIpcMaxBlocks = 256;  // signal slots per rank: [block][rank]
struct IpcPeers {
  const char* data[kIpcMaxRanks];   // every rank's staging region (2 halves of half_bytes)
  uint32_t* sig[kIpcMaxRanks];      // every rank's signal region [kIpcMaxBlocks][kIpcMaxRanks]
  char* mine;                       // this rank's staging region (= data[rank], writable)
  uint32_t* ctr;                    // this rank's per-block epoch counters [kIpcMaxBlocks]
  int* err;                         // this rank's error word (1: a peer never arrived; sticky)
  size_t half_bytes;
};
// buf <- sum over ranks of buf (in place), one kernel: stage, barrier, sum
hipError_t oneshot_all_reduce(const IpcPeers& p, int rank, int world, int64_t n, bool bf16, void* buf, int blocks,
                              hipStream_t s);

}  // namespace ldnn
