// pybind11 bindings of the ldnn gfx950 kernels (module `_C`).
//
// Thin, allocation-free wrappers: every op writes into caller-provided
// tensors and launches on the CURRENT HIP stream, so the Python layer can
// pre-allocate its buffers once and capture whole training steps in hipGraphs.
#include <torch/extension.h>
#include <pybind11/stl.h>
#include <vector>
#include <cstring>
#include <string>
#include <mutex>
#include <map>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <rocprofiler-sdk-roctx/roctx.h>
#include "ldnn_kernels.h"

namespace {

// torch on ROCm reports HIP devices as "cuda"; use its masquerading stream/guard API.
hipStream_t cur_stream(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

void check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "ldnn kernel '", what, "' failed: ", hipGetErrorString(e));
}

void check_dev(const at::Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
}

const uint16_t* bf16_ptr(const at::Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }
uint16_t* bf16_mut(const at::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// Leading dimension of a 2-D operand: row stride; the last dim must be dense.
int64_t ld_of(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 2, name, " must be 2-D");
  TORCH_CHECK(t.stride(1) == 1, name, " must have a unit inner stride");
  return t.stride(0);
}

// C = epi(A_op @ B_op)
//   a: if a_kcontig, [M][K] else [K][M];  b: if b_kcontig, [N][K] else [K][N];  c: [M][N]
void gemm(const at::Tensor& a, const at::Tensor& b, const at::Tensor& c_in, bool a_kcontig, bool b_kcontig,
          int64_t epi, const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& aux,
          const c10::optional<at::Tensor>& dbias, double beta, int64_t tile, int64_t splitk, bool direct_epi,
          int64_t variant, const c10::optional<at::Tensor>& ws, const c10::optional<at::Tensor>& cnt,
          const c10::optional<at::Tensor>& mask_out, const c10::optional<at::Tensor>& mask_in,
          const c10::optional<at::Tensor>& head_w, const c10::optional<at::Tensor>& head_part) {
  check_dev(a, at::kBFloat16, "a");
  check_dev(b, at::kBFloat16, "b");
  TORCH_CHECK(c_in.is_cuda() && (c_in.scalar_type() == at::kBFloat16 || c_in.scalar_type() == at::kFloat),
              "c must be a bf16 or fp32 GPU tensor");
  // a 3-D c = [splitk][M][N] receives the split-K partial products of the four-wave
  // kernel, one slab per split (no in-launch combine; sum them with slab_sum)
  const bool slabs = c_in.dim() == 3;
  if (slabs) {
    TORCH_CHECK(c_in.is_contiguous() && c_in.size(0) == splitk && splitk > 1 && epi == ldnn::EPI_NONE &&
                    !ws.has_value() && !dbias.has_value() && beta == 0.0,
                "gemm: slab output needs a dense [splitk][M][N] c, splitk > 1, EPI_NONE, no ws / dbias / beta");
  }
  const at::Tensor c = slabs ? c_in.select(0, 0) : c_in;
  const bool out_f32 = c.scalar_type() == at::kFloat;
  const int64_t lda = ld_of(a, "a"), ldb = ld_of(b, "b"), ldc = ld_of(c, "c");
  const int64_t M = a_kcontig ? a.size(0) : a.size(1);
  const int64_t K = a_kcontig ? a.size(1) : a.size(0);
  const int64_t N = b_kcontig ? b.size(0) : b.size(1);
  const int64_t Kb = b_kcontig ? b.size(1) : b.size(0);
  TORCH_CHECK(K == Kb, "gemm: inner dims differ (", K, " vs ", Kb, ")");
  TORCH_CHECK(c.size(0) == M && c.size(1) == N, "gemm: output shape mismatch");
  // 16-B vector staging: every contiguous extent and row stride is a multiple of 8 elements.
  TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0, "gemm: leading dims must be multiples of 8");
  TORCH_CHECK(K % 8 == 0 || (a_kcontig == false && b_kcontig == false), "gemm: K must be a multiple of 8");
  TORCH_CHECK(N % 8 == 0, "gemm: N must be a multiple of 8");
  TORCH_CHECK(a_kcontig || M % 8 == 0, "gemm: M must be a multiple of 8 for a k-strided A");
  TORCH_CHECK(aligned16(a.data_ptr()) && aligned16(b.data_ptr()) && aligned16(c.data_ptr()),
              "gemm: operands must be 16-byte aligned");
  ldnn::GemmParams p{};
  p.A = bf16_ptr(a);
  p.B = bf16_ptr(b);
  p.C = c.data_ptr();
  p.M = (int)M;
  p.N = (int)N;
  p.K = (int)K;
  p.lda = (int)lda;
  p.ldb = (int)ldb;
  p.ldc = (int)ldc;
  p.beta = (float)beta;
  p.direct_epi = direct_epi ? 1 : 0;
  p.variant = (int)variant;
  if (epi == ldnn::EPI_BIAS || epi == ldnn::EPI_BIAS_RELU || epi == ldnn::EPI_BIAS_SIGMOID ||
      epi == ldnn::EPI_BIAS_RELU_MASK) {
    TORCH_CHECK(bias.has_value(), "gemm: bias epilogue needs a bias tensor");
    check_dev(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->is_contiguous() && bias->numel() >= N && aligned16(bias->data_ptr()), "gemm: bad bias");
    p.bias = bias->data_ptr<float>();
  }
  bool force_q = slabs;
  if (mask_out.has_value() || mask_in.has_value()) {
    // ReLU bit masks (four-wave kernel): the forward writes them, the dgrad reads them
    const at::Tensor& mk = mask_out.has_value() ? *mask_out : *mask_in;
    check_dev(mk, at::kByte, "mask");
    TORCH_CHECK(!(mask_out.has_value() && mask_in.has_value()), "gemm: mask_out and mask_in are exclusive");
    TORCH_CHECK(mk.dim() == 2 && mk.size(0) == M && mk.size(1) * 8 >= N && mk.stride(1) == 1, "gemm: bad mask shape");
    TORCH_CHECK(!out_f32 && (mask_out.has_value() ? epi == ldnn::EPI_BIAS_RELU : epi == ldnn::EPI_DRELU),
                "gemm: mask_out goes with EPI_BIAS_RELU, mask_in with EPI_DRELU (bf16 out)");
    p.ldmask = (int)mk.stride(0);
    if (mask_out.has_value()) {
      p.mask_out = mk.data_ptr<uint8_t>();
      epi = ldnn::EPI_BIAS_RELU_MASK;
    } else {
      p.mask_in = mk.data_ptr<uint8_t>();
      epi = ldnn::EPI_DRELU_MASK;
    }
    force_q = true;
  }
  if (head_w.has_value() || head_part.has_value()) {
    // bias + ReLU forward with the classifier head's partial logits (EPI_BIAS_RELU_HEAD)
    TORCH_CHECK(head_w.has_value() && head_part.has_value(), "gemm: head_w and head_part go together");
    TORCH_CHECK(epi == ldnn::EPI_BIAS_RELU && !out_f32 && a_kcontig && b_kcontig && !slabs && !dbias.has_value() &&
                    !mask_out.has_value() && !mask_in.has_value() && splitk <= 1 && beta == 0.0,
                "gemm: head partials need EPI_BIAS_RELU, bf16 out, k-contiguous operands, no split-K / masks / dbias");
    check_dev(*head_w, at::kBFloat16, "head_w");
    check_dev(*head_part, at::kFloat, "head_part");
    TORCH_CHECK(head_w->dim() == 2 && head_w->size(0) == 16 && head_w->size(1) >= N && head_w->stride(1) == 1 &&
                    head_w->stride(0) % 4 == 0 && ((uintptr_t)head_w->data_ptr() & 7) == 0,
                "gemm: head_w must be [16][>= N] bf16 (classes zero-padded to 16), 8-B aligned rows");
    TORCH_CHECK(head_part->is_contiguous() && head_part->dim() == 3 && head_part->size(0) == (N + 255) / 256 &&
                    head_part->size(1) == M && head_part->size(2) == 16 && aligned16(head_part->data_ptr()),
                "gemm: head_part must be a dense [ceil(N / 256)][M][16] fp32 tensor");
    p.head_w = bf16_ptr(*head_w);
    p.ldhw = (int)head_w->stride(0);
    p.head_part = head_part->data_ptr<float>();
    epi = ldnn::EPI_BIAS_RELU_HEAD;
    force_q = true;
  }
  if (epi == ldnn::EPI_DRELU || epi == ldnn::EPI_DSIGMOID) {
    TORCH_CHECK(aux.has_value(), "gemm: derivative epilogue needs the saved activation");
    check_dev(*aux, at::kBFloat16, "aux");
    TORCH_CHECK(aux->size(0) == M && aux->size(1) == N, "gemm: aux shape mismatch");
    p.ldaux = (int)ld_of(*aux, "aux");
    TORCH_CHECK(p.ldaux % 4 == 0 && aligned16(aux->data_ptr()), "gemm: bad aux layout");
    p.aux = bf16_ptr(*aux);
  }
  if (dbias.has_value()) {
    check_dev(*dbias, at::kFloat, "dbias");
    TORCH_CHECK(dbias->is_contiguous() && dbias->numel() >= N, "gemm: bad dbias");
    TORCH_CHECK(!(epi == ldnn::EPI_BIAS || epi == ldnn::EPI_BIAS_RELU || epi == ldnn::EPI_BIAS_SIGMOID ||
                  epi == ldnn::EPI_BIAS_RELU_MASK),
                "gemm: dbias (output column sums) goes with the dgrad / plain epilogues, not a bias forward");
    p.dbias = dbias->data_ptr<float>();
  }
  const bool skinny_ok = a_kcontig && b_kcontig && !out_f32 && N <= 64 && !dbias.has_value() && beta == 0.0 &&
                         (epi == ldnn::EPI_NONE || epi == ldnn::EPI_BIAS || epi == ldnn::EPI_BIAS_RELU ||
                          epi == ldnn::EPI_BIAS_SIGMOID);
  if (force_q) {  // masks / slab output exist only in the four-wave kernel
    TORCH_CHECK(tile == 0 || tile == 256, "gemm: masks / slab output need tile 256");
    tile = 256;
    if ((variant & 255) < 32) variant = (variant & ~255) | 32;
    p.variant = (int)variant;
  }
  if (slabs) {
    p.splitk = (int)splitk;
    p.c_split_stride = M * ldc;
    TORCH_CHECK(c_in.stride(0) == M * ldc, "gemm: slab stride");
  }
  if (tile == 0) tile = skinny_ok && K >= 256 ? 16 : ldnn::gemm_pick_tile(p.M, p.N, p.K, out_f32);
  TORCH_CHECK(tile == 16 || tile == 128 || tile == 256, "gemm: tile must be 0 (auto), 16 (skinny-N), 128 or 256");
  c10::hip::HIPGuardMasqueradingAsCUDA g(a.device());
  if (tile == 16) {
    TORCH_CHECK(skinny_ok, "gemm: the skinny-N kernel needs k-contiguous operands, bf16 out, N <= 64");
    check(ldnn::gemm_skinny_n(p, (int)epi, cur_stream(a)), "gemm_skinny_n");
    return;
  }
  // variant (low byte): 0 = auto (the four-wave gemm_q kernel where it wins, else k256),
  // 1 = gemm.hip k256, 2/3 = k256 ring experiments, 32.. = gemm_q
  if (tile == 256 && (variant & 255) == 0 && ldnn::gemm_q_preferred(p.M, p.N, p.K)) {
    variant |= 32;
    p.variant = (int)variant;
  }
  TORCH_CHECK(!(tile == 256 && (variant & 255) >= 4 && (variant & 255) < 32), "gemm: unknown variant");
  if (tile == 256 && (variant & 255) >= 32) {  // four-wave kernel (gemm_q.hip)
    if (splitk > 1 && !slabs) {
      TORCH_CHECK(ws.has_value() && cnt.has_value(), "gemm: gemm_q's in-launch split-K needs ws and cnt");
      check_dev(*ws, at::kFloat, "ws");
      check_dev(*cnt, at::kInt, "cnt");
      TORCH_CHECK(ws->is_contiguous() && (size_t)ws->numel() * 4 >= ldnn::gemm_q_ws_bytes(p.M, p.N, (int)splitk),
                  "gemm: split-K workspace too small");
      TORCH_CHECK(cnt->is_contiguous() && cnt->numel() >= ldnn::gemm_q_tiles(p.M, p.N), "gemm: too few counters");
      p.splitk = (int)splitk;
      p.ws = ws->data_ptr<float>();
      p.cnt = cnt->data_ptr<int>();
    }
    check(ldnn::gemm_q(p, a_kcontig, b_kcontig, (int)epi, out_f32, cur_stream(a)), "gemm_q");
    return;
  }
  if (ws.has_value() || cnt.has_value()) {
    // in-launch split-K combine: explicit split count, any epilogue, deterministic
    TORCH_CHECK(ws.has_value() && cnt.has_value() && tile == 128 && splitk > 1,
                "gemm: ws/cnt (split-K combine) need tile=128 and splitk > 1");
    check_dev(*ws, at::kFloat, "ws");
    check_dev(*cnt, at::kInt, "cnt");
    TORCH_CHECK(ws->is_contiguous() && (size_t)ws->numel() * 4 >= ldnn::gemm_splitk_ws_bytes(p.M, p.N, (int)splitk),
                "gemm: split-K workspace too small");
    TORCH_CHECK(cnt->is_contiguous() && cnt->numel() >= ldnn::gemm_tiles128(p.M, p.N), "gemm: too few counters");
    TORCH_CHECK(aligned16(ws->data_ptr()), "gemm: workspace alignment");
    p.splitk = (int)splitk;
    p.ws = ws->data_ptr<float>();
    p.cnt = cnt->data_ptr<int>();
  } else if (tile == 128 && out_f32 && epi == ldnn::EPI_NONE && !dbias.has_value() && (beta == 0.0 || beta == 1.0)) {
    p.splitk = splitk > 0 ? (int)splitk : ldnn::gemm_pick_splitk(p.M, p.N, p.K);
  }
  check(ldnn::gemm_bf16_tile(p, a_kcontig, b_kcontig, (int)epi, out_f32, (int)tile, cur_stream(a)), "gemm");
}

// The fused-optimizer state of a weight block `master` (fp32 storage; m / v / shadow in
// the same layout) -> OptEpi; returns the EPI_OPT_* epilogue of `kind` ("sgd" | "adam" | "adamw").
int opt_epi_of(ldnn::OptEpi& o, const at::Tensor& master, const std::string& kind,
               const c10::optional<at::Tensor>& m, const c10::optional<at::Tensor>& v,
               const c10::optional<at::Tensor>& shadow, const at::Tensor& hp, double grad_scale, double momentum,
               double dampening, double weight_decay, bool nesterov, double beta1, double beta2, double eps,
               const char* who) {
  check_dev(master, at::kFloat, "master");
  check_dev(hp, at::kFloat, "hp");
  auto same = [&](const c10::optional<at::Tensor>& t, const char* name) -> float* {
    if (!t.has_value()) return nullptr;
    check_dev(*t, at::kFloat, name);
    TORCH_CHECK(t->sizes() == master.sizes() && t->strides() == master.strides(), who, ": ", name, " layout");
    TORCH_CHECK(aligned16(t->data_ptr()), who, ": ", name, " alignment");
    return t->data_ptr<float>();
  };
  o = ldnn::OptEpi{};
  o.master = master.data_ptr<float>();
  o.m = same(m, "m");
  o.v = same(v, "v");
  if (shadow.has_value()) {
    check_dev(*shadow, at::kBFloat16, "shadow");
    TORCH_CHECK(shadow->sizes() == master.sizes() && shadow->strides() == master.strides(), who, ": shadow layout");
    TORCH_CHECK(((uintptr_t)shadow->data_ptr() & 7) == 0, who, ": shadow alignment");
    o.shadow = bf16_mut(*shadow);
  }
  o.hp = hp.data_ptr<float>();
  o.grad_scale = (float)grad_scale;
  o.momentum = (float)momentum;
  o.dampening = (float)dampening;
  o.weight_decay = (float)weight_decay;
  o.nesterov = nesterov ? 1 : 0;
  o.beta1 = (float)beta1;
  o.beta2 = (float)beta2;
  o.eps = (float)eps;
  if (kind == "sgd") {
    TORCH_CHECK(momentum == 0.0 || o.m, who, ": SGD momentum needs its buffer");
    return ldnn::EPI_OPT_SGD;
  }
  if (kind == "adam" || kind == "adamw") {
    o.decoupled = kind == "adamw" ? 1 : 0;
    TORCH_CHECK(o.m && o.v, who, ": Adam needs exp_avg and exp_avg_sq");
    return ldnn::EPI_OPT_ADAM;
  }
  TORCH_CHECK(false, who, ": unknown optimizer ", kind);
  return -1;
}

// Weight-gradient GEMM whose epilogue applies SGD / Adam to `master` (fp32
// [M][N] storage, the layout of the gradient it replaces) and refreshes the bf16
// shadow: the gradient never goes to HBM.  kind: "sgd" | "adam" | "adamw".
void gemm_opt(const at::Tensor& a, const at::Tensor& b, const at::Tensor& master, bool a_kcontig, bool b_kcontig,
              const std::string& kind, const c10::optional<at::Tensor>& m, const c10::optional<at::Tensor>& v,
              const c10::optional<at::Tensor>& shadow, const at::Tensor& hp, double grad_scale, double momentum,
              double dampening, double weight_decay, bool nesterov, double beta1, double beta2, double eps,
              int64_t tile, int64_t splitk, const c10::optional<at::Tensor>& ws,
              const c10::optional<at::Tensor>& cnt) {
  check_dev(a, at::kBFloat16, "a");
  check_dev(b, at::kBFloat16, "b");
  const int64_t lda = ld_of(a, "a"), ldb = ld_of(b, "b"), ldc = ld_of(master, "master");
  const int64_t M = a_kcontig ? a.size(0) : a.size(1);
  const int64_t K = a_kcontig ? a.size(1) : a.size(0);
  const int64_t N = b_kcontig ? b.size(0) : b.size(1);
  TORCH_CHECK((b_kcontig ? b.size(1) : b.size(0)) == K, "gemm_opt: inner dims differ");
  TORCH_CHECK(master.size(0) == M && master.size(1) == N, "gemm_opt: master shape mismatch");
  TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0 && ldc % 4 == 0 && N % 8 == 0, "gemm_opt: leading dims");
  TORCH_CHECK(a_kcontig || M % 8 == 0, "gemm_opt: M must be a multiple of 8 for a k-strided A");
  ldnn::GemmParams p{};
  p.A = bf16_ptr(a);
  p.B = bf16_ptr(b);
  p.C = master.data_ptr();
  p.M = (int)M;
  p.N = (int)N;
  p.K = (int)K;
  p.lda = (int)lda;
  p.ldb = (int)ldb;
  p.ldc = (int)ldc;
  const int epi = opt_epi_of(p.opt, master, kind, m, v, shadow, hp, grad_scale, momentum, dampening, weight_decay,
                             nesterov, beta1, beta2, eps, "gemm_opt");
  TORCH_CHECK(aligned16(a.data_ptr()) && aligned16(b.data_ptr()) && aligned16(master.data_ptr()), "gemm_opt: alignment");
  if (tile == 0) tile = ldnn::gemm_pick_tile(p.M, p.N, p.K, true);
  if (tile == 256 && splitk <= 1 && ldnn::gemm_q_preferred(p.M, p.N, p.K)) {
    // the four-wave kernel (the one the plain wgrad of this shape runs), row-staged update epilogue
    c10::hip::HIPGuardMasqueradingAsCUDA g(a.device());
    check(ldnn::gemm_q(p, a_kcontig, b_kcontig, epi, true, cur_stream(a)), "gemm_opt (gemm_q)");
    return;
  }
  if (splitk > 1) {
    TORCH_CHECK(tile == 128 && ws.has_value() && cnt.has_value(), "gemm_opt: split-K needs the in-launch combine");
    check_dev(*ws, at::kFloat, "ws");
    check_dev(*cnt, at::kInt, "cnt");
    TORCH_CHECK((size_t)ws->numel() * 4 >= ldnn::gemm_splitk_ws_bytes(p.M, p.N, (int)splitk) &&
                    cnt->numel() >= ldnn::gemm_tiles128(p.M, p.N),
                "gemm_opt: split-K workspace too small");
    p.splitk = (int)splitk;
    p.ws = ws->data_ptr<float>();
    p.cnt = cnt->data_ptr<int>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(a.device());
  check(ldnn::gemm_bf16_tile(p, a_kcontig, b_kcontig, epi, true, (int)tile, cur_stream(a)), "gemm_opt");
}

void act_fwd(const at::Tensor& x, const at::Tensor& y, int64_t act) {
  check_dev(x, at::kBFloat16, "x");
  check_dev(y, at::kBFloat16, "y");
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && x.numel() == y.numel(), "act_fwd: bad tensors");
  check(ldnn::act_fwd(bf16_ptr(x), bf16_mut(y), x.numel(), (int)act, cur_stream(x)), "act_fwd");
}

void act_bwd(const at::Tensor& dy, const at::Tensor& y, const at::Tensor& dx, int64_t act) {
  check_dev(dy, at::kBFloat16, "dy");
  check_dev(y, at::kBFloat16, "y");
  check_dev(dx, at::kBFloat16, "dx");
  TORCH_CHECK(dy.is_contiguous() && y.is_contiguous() && dx.is_contiguous(), "act_bwd: non-contiguous");
  TORCH_CHECK(dy.numel() == y.numel() && dx.numel() == y.numel(), "act_bwd: size mismatch");
  check(ldnn::act_bwd(bf16_ptr(dy), bf16_ptr(y), bf16_mut(dx), y.numel(), (int)act, cur_stream(y)), "act_bwd");
}

// the optional ticketed scratch of colsum / act_bwd_colsum: >= cols + 1 zeroed fp32 (kept zero by the kernel)
float* colsum_ws(const c10::optional<at::Tensor>& ws, int64_t cols) {
  if (!ws.has_value()) return nullptr;
  check_dev(*ws, at::kFloat, "ws");
  TORCH_CHECK(ws->is_contiguous() && ws->numel() >= cols + 1, "colsum: ws needs cols + 1 zeroed floats");
  return ws->data_ptr<float>();
}

void colsum(const at::Tensor& x, const at::Tensor& out, bool accumulate, const c10::optional<at::Tensor>& ws) {
  check_dev(x, at::kBFloat16, "x");
  check_dev(out, at::kFloat, "out");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && x.size(1) % 8 == 0, "colsum: x must be [R][C], C%8==0");
  TORCH_CHECK(out.is_contiguous() && out.numel() >= x.size(1), "colsum: bad out");
  check(ldnn::colsum_bf16(bf16_ptr(x), out.data_ptr<float>(), (int)x.size(0), (int)x.size(1), accumulate,
                          cur_stream(x), colsum_ws(ws, x.size(1))),
        "colsum");
}

void act_bwd_colsum(const at::Tensor& dy, const at::Tensor& y, const at::Tensor& dx, const at::Tensor& out,
                    int64_t act, bool accumulate, const c10::optional<at::Tensor>& ws) {
  check_dev(dy, at::kBFloat16, "dy");
  check_dev(y, at::kBFloat16, "y");
  check_dev(dx, at::kBFloat16, "dx");
  check_dev(out, at::kFloat, "out");
  TORCH_CHECK(y.dim() == 2 && y.is_contiguous() && dy.is_contiguous() && dx.is_contiguous() &&
                  out.is_contiguous(), "act_bwd_colsum: tensors must be contiguous, y 2-D");
  TORCH_CHECK(dy.sizes() == y.sizes() && dx.sizes() == y.sizes(), "act_bwd_colsum: size mismatch");
  TORCH_CHECK(y.size(1) % 8 == 0 && out.numel() >= y.size(1), "act_bwd_colsum: cols % 8 != 0 or short out");
  TORCH_CHECK(act == ldnn::ACT_RELU || act == ldnn::ACT_SIGMOID, "act_bwd_colsum: act must be relu/sigmoid");
  check(ldnn::act_bwd_colsum(bf16_ptr(dy), bf16_ptr(y), bf16_mut(dx), out.data_ptr<float>(), (int)y.size(0),
                             (int)y.size(1), (int)act, accumulate, cur_stream(y), colsum_ws(ws, y.size(1))),
        "act_bwd_colsum");
}

void cast_f32_bf16(const at::Tensor& x, const at::Tensor& y) {
  check_dev(x, at::kFloat, "x");
  check_dev(y, at::kBFloat16, "y");
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && x.numel() == y.numel(), "cast: bad tensors");
  check(ldnn::cast_f32_bf16(x.data_ptr<float>(), bf16_mut(y), x.numel(), cur_stream(x)), "cast_f32_bf16");
}

void cast_bf16_f32(const at::Tensor& x, const at::Tensor& y) {
  check_dev(x, at::kBFloat16, "x");
  check_dev(y, at::kFloat, "y");
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && x.numel() == y.numel(), "cast: bad tensors");
  check(ldnn::cast_bf16_f32(bf16_ptr(x), y.data_ptr<float>(), x.numel(), cur_stream(x)), "cast_bf16_f32");
}

void mix3(const at::Tensor& out, const at::Tensor& x, const c10::optional<at::Tensor>& y1,
          const c10::optional<at::Tensor>& y2, double a, double b, double c,
          const c10::optional<at::Tensor>& shadow) {
  check_dev(out, at::kFloat, "out");
  check_dev(x, at::kFloat, "x");
  const int64_t n = out.numel();
  TORCH_CHECK(out.is_contiguous() && x.is_contiguous() && x.numel() == n, "mix3: bad x/out");
  if (y1.has_value() && y1->scalar_type() == at::kBFloat16) {   // bf16 neighbour copies (gossip exchange)
    check_dev(*y1, at::kBFloat16, "y1");
    TORCH_CHECK(y1->is_contiguous() && y1->numel() == n, "mix3: bad y1");
    const uint16_t* q2 = nullptr;
    if (y2.has_value()) {
      check_dev(*y2, at::kBFloat16, "y2");
      TORCH_CHECK(y2->is_contiguous() && y2->numel() == n, "mix3: bad y2");
      q2 = bf16_ptr(*y2);
    }
    uint16_t* sh16 = nullptr;
    if (shadow.has_value()) {
      check_dev(*shadow, at::kBFloat16, "shadow");
      TORCH_CHECK(shadow->is_contiguous() && shadow->numel() == n, "mix3: bad shadow");
      sh16 = bf16_mut(*shadow);
    }
    check(ldnn::mix3_y16(out.data_ptr<float>(), x.data_ptr<float>(), bf16_ptr(*y1), q2, (float)a, (float)b, (float)c, n,
                         sh16, cur_stream(out)),
          "mix3");
    return;
  }
  const float* p1 = nullptr;
  const float* p2 = nullptr;
  if (y1.has_value()) {
    check_dev(*y1, at::kFloat, "y1");
    TORCH_CHECK(y1->is_contiguous() && y1->numel() == n, "mix3: bad y1");
    p1 = y1->data_ptr<float>();
  }
  if (y2.has_value()) {
    TORCH_CHECK(p1 != nullptr, "mix3: y2 without y1");
    check_dev(*y2, at::kFloat, "y2");
    TORCH_CHECK(y2->is_contiguous() && y2->numel() == n, "mix3: bad y2");
    p2 = y2->data_ptr<float>();
  }
  uint16_t* sh = nullptr;
  if (shadow.has_value()) {
    check_dev(*shadow, at::kBFloat16, "shadow");
    TORCH_CHECK(shadow->is_contiguous() && shadow->numel() == n, "mix3: bad shadow");
    sh = bf16_mut(*shadow);
  }
  check(ldnn::mix3_f32(out.data_ptr<float>(), x.data_ptr<float>(), p1, p2, (float)a, (float)b, (float)c, n, sh,
                       cur_stream(out)),
        "mix3");
}

// Self-cleaning [acc0, acc1, counter] of the finalizing softmax-xent, one per
// (device, stream): the kernels leave it zero, so it is zeroed once at creation.
int* xent_fin_ws(const at::Tensor& like) {
  static std::mutex mu;
  static std::map<std::pair<int, int64_t>, at::Tensor> pools;
  const auto key = std::make_pair((int)like.get_device(), (int64_t)cur_stream(like));
  std::lock_guard<std::mutex> lock(mu);
  auto it = pools.find(key);
  if (it == pools.end()) it = pools.emplace(key, at::zeros({4}, like.options().dtype(at::kInt))).first;
  return it->second.data_ptr<int>();
}

void softmax_xent(const at::Tensor& logits, const at::Tensor& labels, const at::Tensor& dlogits,
                  const c10::optional<at::Tensor>& stats, const c10::optional<at::Tensor>& dbias, int64_t num_classes,
                  double grad_scale, const c10::optional<at::Tensor>& loss_out, double loss_scale) {
  check_dev(logits, at::kBFloat16, "logits");
  check_dev(dlogits, at::kBFloat16, "dlogits");
  check_dev(labels, at::kLong, "labels");
  float* st = nullptr;
  if (stats.has_value()) {
    check_dev(*stats, at::kFloat, "stats");
    TORCH_CHECK(stats->numel() >= 2, "xent: stats needs 2 floats");
    st = stats->data_ptr<float>();
  }
  TORCH_CHECK(st != nullptr || loss_out.has_value(), "xent: give stats and/or loss_out");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1 && dlogits.sizes() == logits.sizes() &&
                  dlogits.strides() == logits.strides(),
              "xent: logits/dlogits layout mismatch");
  TORCH_CHECK(labels.is_contiguous() && labels.numel() == logits.size(0), "xent: bad labels");
  // logits may be a [B][C] view of a zero-padded [B][ld] buffer (ld % 8 == 0):
  // the kernel reads C columns and writes all ld columns of dlogits (pad = 0).
  const int64_t ld = logits.stride(0);
  TORCH_CHECK(num_classes <= logits.size(1) && logits.size(1) <= ld, "xent: bad class count / row stride");
  TORCH_CHECK((int64_t)dlogits.storage().nbytes() >= (dlogits.storage_offset() + logits.size(0) * ld) * 2,
              "xent: dlogits storage must hold the padded [B][ld] rows");
  float* db = nullptr;
  if (dbias.has_value()) {
    check_dev(*dbias, at::kFloat, "dbias");
    TORCH_CHECK(dbias->numel() >= ld, "xent: bad dbias");
    db = dbias->data_ptr<float>();
  }
  ldnn::XentFin fin;
  if (loss_out.has_value()) {
    check_dev(*loss_out, at::kFloat, "loss_out");
    TORCH_CHECK(loss_out->numel() >= 2 && loss_out->is_contiguous(), "xent: loss_out needs 2 dense floats");
    int* ws = xent_fin_ws(logits);
    fin.out = loss_out->data_ptr<float>();
    fin.acc = reinterpret_cast<float*>(ws);
    fin.cnt = reinterpret_cast<unsigned*>(ws + 2);
    fin.scale = (float)loss_scale;
  }
  check(ldnn::softmax_xent(bf16_ptr(logits), labels.data_ptr<int64_t>(), bf16_mut(dlogits), st, db,
                           (int)logits.size(0), (int)num_classes, (int)ld, (float)grad_scale, cur_stream(logits),
                           loss_out.has_value() ? &fin : nullptr),
        "softmax_xent");
}

// up to two [begin, end) element ranges of `grad` to clear after the update reads them
ldnn::GradZero grad_zero(const std::vector<std::pair<int64_t, int64_t>>& r, int64_t n) {
  TORCH_CHECK(r.size() <= 2, "optimizer: at most two gradient zero ranges");
  ldnn::GradZero z;
  for (size_t i = 0; i < r.size(); ++i) {
    TORCH_CHECK(0 <= r[i].first && r[i].first <= r[i].second && r[i].second <= n, "optimizer: bad zero range");
    z.zb[i] = r[i].first;
    z.ze[i] = r[i].second;
  }
  return z;
}

void sgd_step(const at::Tensor& param, const at::Tensor& grad, const at::Tensor& mom,
              const c10::optional<at::Tensor>& shadow, const at::Tensor& hp, double grad_scale, double momentum,
              double dampening, double weight_decay, bool nesterov, bool first_step,
              const std::vector<std::pair<int64_t, int64_t>>& zero_ranges, int64_t t_begin,
              const c10::optional<at::Tensor>& t_out) {
  check_dev(param, at::kFloat, "param");
  check_dev(grad, at::kFloat, "grad");
  check_dev(hp, at::kFloat, "hp");
  const int64_t n = param.numel();
  TORCH_CHECK(param.is_contiguous() && grad.is_contiguous() && grad.numel() == n, "sgd: bad param/grad");
  float* mp = nullptr;
  if (momentum != 0.0) {
    check_dev(mom, at::kFloat, "mom");
    TORCH_CHECK(mom.is_contiguous() && mom.numel() == n, "sgd: bad momentum buffer");
    mp = mom.data_ptr<float>();
  }
  uint16_t* sh = nullptr;
  if (shadow.has_value()) {
    check_dev(*shadow, at::kBFloat16, "shadow");
    TORCH_CHECK(shadow->is_contiguous() && shadow->numel() == n, "sgd: bad shadow");
    sh = bf16_mut(*shadow);
  }
  ldnn::SgdParams sp{(float)momentum, (float)dampening, (float)weight_decay, nesterov ? 1 : 0, first_step ? 1 : 0,
                     grad_zero(zero_ranges, n)};
  ldnn::ShadowT tr{};
  if (t_out.has_value()) {
    // t_out [cols][rows] bf16: the transposed shadow of the [rows][cols] matrix at element t_begin
    check_dev(*t_out, at::kBFloat16, "t_out");
    TORCH_CHECK(t_out->dim() == 2 && t_out->is_contiguous() && t_begin >= 0 &&
                    t_begin + t_out->numel() <= n && t_out->size(0) % 64 == 0 && t_out->size(1) % 64 == 0 &&
                    t_begin % 4 == 0 && aligned16(t_out->data_ptr()),
                "sgd: t_out must be a dense [cols][rows] bf16 tensor (multiples of 64) inside the range");
    tr.begin = t_begin;
    tr.rows = (int)t_out->size(1);
    tr.cols = (int)t_out->size(0);
    tr.out = bf16_mut(*t_out);
  }
  check(ldnn::sgd_step(param.data_ptr<float>(), grad.data_ptr<float>(), mp, sh, hp.data_ptr<float>(),
                       (float)grad_scale, sp, n, cur_stream(param), t_out.has_value() ? &tr : nullptr),
        "sgd_step");
}

void adam_step(const at::Tensor& param, const at::Tensor& grad, const at::Tensor& m, const at::Tensor& v,
               const c10::optional<at::Tensor>& shadow, const at::Tensor& hp, double grad_scale, double beta1,
               double beta2, double eps, double weight_decay, bool decoupled,
               const std::vector<std::pair<int64_t, int64_t>>& zero_ranges) {
  check_dev(param, at::kFloat, "param");
  check_dev(grad, at::kFloat, "grad");
  check_dev(m, at::kFloat, "exp_avg");
  check_dev(v, at::kFloat, "exp_avg_sq");
  check_dev(hp, at::kFloat, "hp");
  const int64_t n = param.numel();
  TORCH_CHECK(param.is_contiguous() && grad.is_contiguous() && m.is_contiguous() && v.is_contiguous() &&
                  grad.numel() == n && m.numel() == n && v.numel() == n,
              "adam: bad buffers");
  uint16_t* sh = nullptr;
  if (shadow.has_value()) {
    check_dev(*shadow, at::kBFloat16, "shadow");
    TORCH_CHECK(shadow->is_contiguous() && shadow->numel() == n, "adam: bad shadow");
    sh = bf16_mut(*shadow);
  }
  ldnn::AdamParams ap{(float)beta1, (float)beta2, (float)eps, (float)weight_decay, decoupled ? 1 : 0,
                      grad_zero(zero_ranges, n)};
  check(ldnn::adam_step(param.data_ptr<float>(), grad.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                        sh, hp.data_ptr<float>(), (float)grad_scale, ap, n, cur_stream(param)),
        "adam_step");
}

void head_fwd_xent(const at::Tensor& h, const at::Tensor& W, const at::Tensor& bias, const at::Tensor& labels,
                   const c10::optional<at::Tensor>& logits, const at::Tensor& dlogits, const at::Tensor& stats,
                   int64_t num_classes, double grad_scale, const c10::optional<at::Tensor>& dh,
                   const c10::optional<at::Tensor>& dbias, int64_t dgrad_epi,
                   const c10::optional<at::Tensor>& dbias_ws, int64_t dgrad_mode) {
  check_dev(h, at::kBFloat16, "h");
  check_dev(W, at::kBFloat16, "W");
  check_dev(bias, at::kFloat, "bias");
  check_dev(labels, at::kLong, "labels");
  check_dev(dlogits, at::kBFloat16, "dlogits");
  check_dev(stats, at::kFloat, "stats");
  TORCH_CHECK(h.dim() == 2 && W.dim() == 2 && dlogits.dim() == 2, "head: 2-D operands");
  const int64_t B = h.size(0), K = h.size(1), ld = dlogits.size(1);
  TORCH_CHECK(h.stride(1) == 1 && W.stride(1) == 1 && W.size(1) == K, "head: h / W must be k-contiguous, same K");
  TORCH_CHECK(dlogits.is_contiguous() && dlogits.size(0) == B && ld % 16 == 0 && ld <= 64,
              "head: dlogits must be a contiguous [B][ld] buffer, ld a multiple of 16 <= 64");
  TORCH_CHECK(W.size(0) <= ld && num_classes <= W.size(0), "head: W rows must cover the classes, <= ld");
  TORCH_CHECK(bias.is_contiguous() && bias.numel() >= ld, "head: bias must be padded to ld");
  TORCH_CHECK(labels.is_contiguous() && labels.numel() == B, "head: bad labels");
  TORCH_CHECK(stats.is_contiguous() && stats.numel() >= 2 * ((B + 15) / 16), "head: stats needs 2 floats per 16 rows");
  TORCH_CHECK(h.stride(0) % 8 == 0 && W.stride(0) % 8 == 0 && K % 8 == 0 && aligned16(h.data_ptr()) &&
                  aligned16(W.data_ptr()) && aligned16(bias.data_ptr()),
              "head: 16-B aligned rows required");
  ldnn::HeadParams p{};
  p.h = bf16_ptr(h);
  p.W = bf16_ptr(W);
  p.bias = bias.data_ptr<float>();
  p.labels = labels.data_ptr<int64_t>();
  if (logits.has_value()) {
    check_dev(*logits, at::kBFloat16, "logits");
    TORCH_CHECK(logits->is_contiguous() && logits->sizes() == dlogits.sizes(), "head: logits like dlogits");
    p.logits = bf16_mut(*logits);
  }
  p.dlogits = bf16_mut(dlogits);
  p.stats = stats.data_ptr<float>();
  p.B = (int)B;
  p.K = (int)K;
  p.C = (int)num_classes;
  p.ld = (int)ld;
  p.ldh = (int)h.stride(0);
  p.ldw = (int)W.stride(0);
  p.ldw_rows = (int)W.size(0);
  p.grad_scale = (float)grad_scale;
  if (dh.has_value()) {
    check_dev(*dh, at::kBFloat16, "dh");
    TORCH_CHECK(dh->dim() == 2 && dh->size(0) == B && dh->size(1) == K && dh->stride(1) == 1 &&
                    dh->stride(0) % 8 == 0 && aligned16(dh->data_ptr()),
                "head: dh must be [B][K] with 16-B aligned rows");
    if (dgrad_mode < 0) dgrad_mode = ld == 16 ? 0 : 1;  // auto: the streaming dgrad where it applies
    TORCH_CHECK(dgrad_mode >= 0 && dgrad_mode <= 2, "head: dgrad_mode must be -1 (auto), 0, 1 or 2");
    TORCH_CHECK(dgrad_mode != 0 || ld == 16, "head: the streaming dgrad (mode 0) needs ld == 16");
    TORCH_CHECK(dgrad_mode == 0 || K <= ldnn::head_dgrad_max_k(), "head: fused dgrad needs K <= ",
                ldnn::head_dgrad_max_k());
    p.dgrad_mode = (int)dgrad_mode;
    TORCH_CHECK(dgrad_epi == ldnn::EPI_NONE || dgrad_epi == ldnn::EPI_DRELU || dgrad_epi == ldnn::EPI_DSIGMOID,
                "head: dgrad_epi must be EPI_NONE / EPI_DRELU / EPI_DSIGMOID");
    p.dh = bf16_mut(*dh);
    p.lddh = (int)dh->stride(0);
    p.dgrad_epi = (int)dgrad_epi;
    if (dbias.has_value()) {
      check_dev(*dbias, at::kFloat, "dbias");
      TORCH_CHECK(dbias->is_contiguous() && dbias->numel() >= K && aligned16(dbias->data_ptr()),
                  "head: dbias must hold K floats, 16-B aligned");
      p.dbias = dbias->data_ptr<float>();
      if (dgrad_mode == 1 || dgrad_mode == 2) {  // the fused modes reduce per-workgroup slabs
        TORCH_CHECK(dbias_ws.has_value(), "head: dbias needs dbias_ws (head_dgrad_ws_floats(B, K) fp32)");
        check_dev(*dbias_ws, at::kFloat, "dbias_ws");
        TORCH_CHECK(dbias_ws->is_contiguous() &&
                        dbias_ws->numel() >= (int64_t)ldnn::head_dgrad_ws_floats((int)B, (int)K) &&
                        aligned16(dbias_ws->data_ptr()),
                    "head: dbias_ws too small");
        p.dbias_ws = dbias_ws->data_ptr<float>();
      }
    }
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(h.device());
  check(ldnn::head_fwd_xent(p, cur_stream(h)), "head_fwd_xent");
}

// Softmax-xent from the partial logits of an EPI_BIAS_RELU_HEAD forward (gemm head_part)
void head_xent_parts(const at::Tensor& parts, const at::Tensor& bias, const at::Tensor& labels,
                     const c10::optional<at::Tensor>& logits, const at::Tensor& dlogits, const at::Tensor& stats,
                     int64_t num_classes, double grad_scale) {
  check_dev(parts, at::kFloat, "parts");
  check_dev(bias, at::kFloat, "bias");
  check_dev(labels, at::kLong, "labels");
  check_dev(dlogits, at::kBFloat16, "dlogits");
  check_dev(stats, at::kFloat, "stats");
  TORCH_CHECK(parts.dim() == 3 && parts.is_contiguous() && parts.size(2) == 16 && aligned16(parts.data_ptr()),
              "head_xent_parts: parts must be a dense [nparts][B][16] fp32 tensor");
  const int64_t B = parts.size(1);
  TORCH_CHECK(dlogits.is_contiguous() && dlogits.dim() == 2 && dlogits.size(0) == B && dlogits.size(1) == 16,
              "head_xent_parts: dlogits must be a contiguous [B][16] buffer");
  TORCH_CHECK(num_classes >= 1 && num_classes <= 16, "head_xent_parts: 1..16 classes");
  TORCH_CHECK(bias.is_contiguous() && bias.numel() >= 16 && aligned16(bias.data_ptr()), "head_xent_parts: bias padded to 16");
  TORCH_CHECK(labels.is_contiguous() && labels.numel() == B, "head_xent_parts: bad labels");
  TORCH_CHECK(stats.is_contiguous() && stats.numel() >= 2 * ((B + 15) / 16), "head_xent_parts: stats needs 2 floats per 16 rows");
  ldnn::HeadParams p{};
  p.bias = bias.data_ptr<float>();
  p.labels = labels.data_ptr<int64_t>();
  if (logits.has_value()) {
    check_dev(*logits, at::kBFloat16, "logits");
    TORCH_CHECK(logits->is_contiguous() && logits->sizes() == dlogits.sizes(), "head_xent_parts: logits like dlogits");
    p.logits = bf16_mut(*logits);
  }
  p.dlogits = bf16_mut(dlogits);
  p.stats = stats.data_ptr<float>();
  p.B = (int)B;
  p.C = (int)num_classes;
  p.ld = 16;
  p.grad_scale = (float)grad_scale;
  c10::hip::HIPGuardMasqueradingAsCUDA g(parts.device());
  check(ldnn::head_xent_parts(p, parts.data_ptr<float>(), (int)parts.size(0), cur_stream(parts)), "head_xent_parts");
}

// dh = (dlogits W) * act'(h) and dbias += column sums of dh (the streaming head dgrad alone)
void head_dgrad_stream(const at::Tensor& h, const at::Tensor& W, const at::Tensor& dlogits, const at::Tensor& dh,
                       const c10::optional<at::Tensor>& dbias, int64_t dgrad_epi) {
  check_dev(h, at::kBFloat16, "h");
  check_dev(W, at::kBFloat16, "W");
  check_dev(dlogits, at::kBFloat16, "dlogits");
  check_dev(dh, at::kBFloat16, "dh");
  const int64_t B = h.size(0), K = h.size(1);
  TORCH_CHECK(h.dim() == 2 && h.stride(1) == 1 && h.stride(0) % 8 == 0 && K % 8 == 0 && aligned16(h.data_ptr()),
              "head_dgrad_stream: h must be [B][K] with 16-B aligned rows");
  TORCH_CHECK(W.dim() == 2 && W.size(0) <= 16 && W.size(1) == K && W.stride(1) == 1 && W.stride(0) % 8 == 0 &&
                  aligned16(W.data_ptr()),
              "head_dgrad_stream: W must be [<= 16][K] with 16-B aligned rows");
  TORCH_CHECK(dlogits.is_contiguous() && dlogits.dim() == 2 && dlogits.size(0) == B && dlogits.size(1) == 16,
              "head_dgrad_stream: dlogits must be a contiguous [B][16] buffer");
  TORCH_CHECK(dh.dim() == 2 && dh.size(0) == B && dh.size(1) == K && dh.stride(1) == 1 && dh.stride(0) % 8 == 0 &&
                  aligned16(dh.data_ptr()),
              "head_dgrad_stream: dh must be [B][K] with 16-B aligned rows");
  TORCH_CHECK(dgrad_epi == ldnn::EPI_NONE || dgrad_epi == ldnn::EPI_DRELU || dgrad_epi == ldnn::EPI_DSIGMOID,
              "head_dgrad_stream: dgrad_epi must be EPI_NONE / EPI_DRELU / EPI_DSIGMOID");
  ldnn::HeadParams p{};
  p.h = bf16_ptr(h);
  p.W = bf16_ptr(W);
  p.dlogits = bf16_mut(dlogits);
  p.B = (int)B;
  p.K = (int)K;
  p.ld = 16;
  p.ldh = (int)h.stride(0);
  p.ldw = (int)W.stride(0);
  p.ldw_rows = (int)W.size(0);
  p.dh = bf16_mut(dh);
  p.lddh = (int)dh.stride(0);
  p.dgrad_epi = (int)dgrad_epi;
  if (dbias.has_value()) {
    check_dev(*dbias, at::kFloat, "dbias");
    TORCH_CHECK(dbias->is_contiguous() && dbias->numel() >= K, "head_dgrad_stream: bad dbias");
    p.dbias = dbias->data_ptr<float>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(h.device());
  check(ldnn::head_dgrad_stream(p, cur_stream(h)), "head_dgrad_stream");
}

// the head's dgrad (as head_dgrad_stream) and wgrad (dW / db accumulated, pre-cleared) in one pass
void head_bwd(const at::Tensor& h, const at::Tensor& W, const at::Tensor& dlogits, const at::Tensor& dh,
              const at::Tensor& dW, const c10::optional<at::Tensor>& dbias, int64_t dgrad_epi,
              const c10::optional<at::Tensor>& db) {
  check_dev(h, at::kBFloat16, "h");
  check_dev(W, at::kBFloat16, "W");
  check_dev(dlogits, at::kBFloat16, "dlogits");
  check_dev(dh, at::kBFloat16, "dh");
  check_dev(dW, at::kFloat, "dW");
  const int64_t B = h.size(0), K = h.size(1);
  TORCH_CHECK(h.dim() == 2 && h.stride(1) == 1 && h.stride(0) % 8 == 0 && K % 64 == 0 && aligned16(h.data_ptr()),
              "head_bwd: h must be [B][K] with K % 64 == 0 and 16-B aligned rows");
  TORCH_CHECK(W.dim() == 2 && W.size(0) <= 16 && W.size(1) == K && W.stride(1) == 1, "head_bwd: W must be [<= 16][K]");
  TORCH_CHECK(dlogits.is_contiguous() && dlogits.dim() == 2 && dlogits.size(0) == B && dlogits.size(1) == 16 &&
                  aligned16(dlogits.data_ptr()),
              "head_bwd: dlogits must be a contiguous [B][16] buffer");
  TORCH_CHECK(dh.dim() == 2 && dh.size(0) == B && dh.size(1) == K && dh.stride(1) == 1 && dh.stride(0) % 8 == 0 &&
                  aligned16(dh.data_ptr()),
              "head_bwd: dh must be [B][K] with 16-B aligned rows");
  TORCH_CHECK(dgrad_epi == ldnn::EPI_NONE || dgrad_epi == ldnn::EPI_DRELU, "head_bwd: dgrad_epi must be EPI_NONE / EPI_DRELU");
  TORCH_CHECK(dW.dim() == 2 && dW.size(1) == K && dW.size(0) <= 16 && dW.stride(1) == 1, "head_bwd: dW must be [<= 16][K]");
  ldnn::HeadParams p{};
  p.h = bf16_ptr(h);
  p.W = bf16_ptr(W);
  p.dlogits = bf16_mut(dlogits);
  p.B = (int)B;
  p.K = (int)K;
  p.ld = 16;
  p.ldh = (int)h.stride(0);
  p.ldw = (int)W.stride(0);
  p.ldw_rows = (int)W.size(0);
  p.dh = bf16_mut(dh);
  p.lddh = (int)dh.stride(0);
  p.dgrad_epi = (int)dgrad_epi;
  p.dW = dW.data_ptr<float>();
  p.lddw = (int)dW.stride(0);
  p.nrows_w = (int)dW.size(0);
  if (dbias.has_value()) {
    check_dev(*dbias, at::kFloat, "dbias");
    TORCH_CHECK(dbias->is_contiguous() && dbias->numel() >= K, "head_bwd: bad dbias");
    p.dbias = dbias->data_ptr<float>();
  }
  if (db.has_value()) {
    check_dev(*db, at::kFloat, "db");
    TORCH_CHECK(db->is_contiguous() && db->numel() >= dW.size(0), "head_bwd: bad db");
    p.db = db->data_ptr<float>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(h.device());
  check(ldnn::head_bwd(p, cur_stream(h)), "head_bwd");
}

void head_wgrad(const at::Tensor& dz, const at::Tensor& h, const at::Tensor& dW, const c10::optional<at::Tensor>& db,
                int64_t splits) {
  check_dev(dz, at::kBFloat16, "dz");
  check_dev(h, at::kBFloat16, "h");
  check_dev(dW, at::kFloat, "dW");
  const int64_t B = h.size(0), K = h.size(1), ld = dz.size(1);
  TORCH_CHECK(dz.is_contiguous() && dz.size(0) == B && ld % 16 == 0 && ld <= 64, "head_wgrad: dz [B][ld], ld % 16 == 0");
  TORCH_CHECK(h.stride(1) == 1 && h.stride(0) % 8 == 0 && K % 8 == 0 && aligned16(h.data_ptr()), "head_wgrad: bad h");
  TORCH_CHECK(dW.dim() == 2 && dW.size(1) == K && dW.stride(1) == 1 && dW.size(0) <= ld && dW.stride(0) % 4 == 0 &&
                  aligned16(dW.data_ptr()),
              "head_wgrad: dW must be [rows <= ld][K] with 16-B aligned rows");
  ldnn::HeadWgradParams p{};
  p.dz = bf16_ptr(dz);
  p.h = bf16_ptr(h);
  p.dW = dW.data_ptr<float>();
  if (db.has_value()) {
    check_dev(*db, at::kFloat, "db");
    TORCH_CHECK(db->is_contiguous() && db->numel() >= dW.size(0), "head_wgrad: bad db");
    p.db = db->data_ptr<float>();
  }
  p.B = (int)B;
  p.K = (int)K;
  p.ld = (int)ld;
  p.ldh = (int)h.stride(0);
  p.lddw = (int)dW.stride(0);
  p.nrows = (int)dW.size(0);
  c10::hip::HIPGuardMasqueradingAsCUDA g(h.device());
  check(ldnn::head_wgrad(p, (int)splits, cur_stream(h)), "head_wgrad");
}

void bump_step(const at::Tensor& hp) {
  check_dev(hp, at::kFloat, "hp");
  check(ldnn::bump_step(hp.data_ptr<float>(), cur_stream(hp)), "bump_step");
}

void synth_normal(const at::Tensor& x, int64_t seed, double stddev) {
  check_dev(x, at::kBFloat16, "x");
  TORCH_CHECK(x.is_contiguous(), "synth_normal: x must be contiguous");
  check(ldnn::synth_normal_bf16(bf16_mut(x), x.numel(), (uint64_t)seed, (float)stddev, cur_stream(x)),
        "synth_normal");
}

void synth_labels(const at::Tensor& y, int64_t classes, int64_t seed) {
  check_dev(y, at::kLong, "y");
  TORCH_CHECK(y.is_contiguous(), "synth_labels: y must be contiguous");
  check(ldnn::synth_labels(y.data_ptr<int64_t>(), y.numel(), (int)classes, (uint64_t)seed, cur_stream(y)),
        "synth_labels");
}

// out[b] = normalise(augment(images[index[b]])), see augment.hip / data/autoaugment.py
void augment_batch(const at::Tensor& images, const at::Tensor& index, const at::Tensor& out, const at::Tensor& a,
                   const at::Tensor& b, int64_t seed, int64_t mode, int64_t pad, int64_t fixed_op, int64_t fixed_bin,
                   int64_t fixed_sign, const std::vector<double>& mags, const std::vector<double>& rot_cos,
                   const std::vector<double>& rot_sin, const std::vector<int64_t>& pol_op,
                   const std::vector<double>& pol_prob, const std::vector<int64_t>& pol_bin,
                   const std::vector<int64_t>& signed_op) {
  check_dev(images, at::kByte, "images");
  check_dev(index, at::kLong, "index");
  check_dev(a, at::kFloat, "a");
  check_dev(b, at::kFloat, "b");
  TORCH_CHECK(out.is_cuda() && (out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat),
              "augment: out must be a bf16 or fp32 GPU tensor");
  TORCH_CHECK(images.dim() == 4 && images.is_contiguous(), "augment: images must be a dense [N][C][H][W] tensor");
  TORCH_CHECK(index.dim() == 1 && index.is_contiguous(), "augment: index must be a dense 1-D tensor");
  const int64_t B = index.numel(), C = images.size(1), H = images.size(2), W = images.size(3);
  TORCH_CHECK(out.is_contiguous() && out.dim() == 4 && out.size(0) == B && out.size(1) == C && out.size(2) == H &&
              out.size(3) == W, "augment: out must be a dense [B][C][H][W] tensor");
  TORCH_CHECK(a.numel() >= C && b.numel() >= C, "augment: a / b need one value per channel");
  TORCH_CHECK(C >= 1 && C <= 3 && C * H * W <= ldnn::kAugMaxPixels, "augment: images of ", C, "x", H, "x", W,
              " do not fit the LDS-resident kernel");
  TORCH_CHECK((int64_t)mags.size() == ldnn::kAugOps * ldnn::kAugBins && (int64_t)rot_cos.size() == ldnn::kAugBins &&
              (int64_t)rot_sin.size() == ldnn::kAugBins && (int64_t)signed_op.size() == ldnn::kAugOps,
              "augment: bad magnitude tables");
  TORCH_CHECK(pol_op.size() == pol_prob.size() && pol_op.size() == pol_bin.size() && pol_op.size() % 2 == 0 &&
              (int64_t)pol_op.size() <= ldnn::kAugPolicySlots, "augment: bad policy table");
  TORCH_CHECK(fixed_op < ldnn::kAugOps && fixed_bin < ldnn::kAugBins, "augment: bad fixed op");
  ldnn::AugParams p{};
  p.images = images.data_ptr<uint8_t>();
  p.index = index.data_ptr<int64_t>();
  p.out = out.data_ptr();
  p.a = a.data_ptr<float>();
  p.b = b.data_ptr<float>();
  p.n_images = images.size(0);
  p.B = (int)B;
  p.C = (int)C;
  p.H = (int)H;
  p.W = (int)W;
  p.seed = (uint64_t)seed;
  p.mode = (int)mode;
  p.pad = (int)pad;
  p.fixed_op = (int)fixed_op;
  p.fixed_bin = (int)fixed_bin;
  p.fixed_sign = (int)fixed_sign;
  p.n_policies = (int)(pol_op.size() / 2);
  for (int o = 0; o < ldnn::kAugOps; ++o) {
    for (int k = 0; k < ldnn::kAugBins; ++k) p.mags[o][k] = (float)mags[o * ldnn::kAugBins + k];
    p.signed_op[o] = (int)signed_op[o];
  }
  for (int k = 0; k < ldnn::kAugBins; ++k) {
    p.rot_cos[k] = (float)rot_cos[k];
    p.rot_sin[k] = (float)rot_sin[k];
  }
  for (size_t i = 0; i < pol_op.size(); ++i) {
    p.pol_op[i] = (int)pol_op[i];
    p.pol_prob[i] = (float)pol_prob[i];
    p.pol_bin[i] = (int)pol_bin[i];
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(images.device());
  check(ldnn::augment_batch(p, out.scalar_type() == at::kFloat, cur_stream(images)), "augment_batch");
}

ldnn::ConvShape conv_shape(const at::Tensor& x, const at::Tensor& w, const at::Tensor& y, int64_t stride,
                           int64_t pad) {
  // x [N][H][W][C], w [K][R][S][C], y [N][P][Q][K]  (bf16, dense, C % 8 == K % 8 == 0)
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && y.dim() == 4, "conv: NHWC / KRSC 4-D tensors expected");
  TORCH_CHECK(x.is_contiguous() && w.is_contiguous() && y.is_contiguous(), "conv: tensors must be dense NHWC/KRSC");
  ldnn::ConvShape s{};
  s.N = (int)x.size(0); s.H = (int)x.size(1); s.W = (int)x.size(2); s.C = (int)x.size(3);
  s.K = (int)w.size(0); s.R = (int)w.size(1); s.S = (int)w.size(2);
  s.P = (int)y.size(1); s.Q = (int)y.size(2);
  s.stride = (int)stride; s.pad = (int)pad;
  TORCH_CHECK(w.size(3) == s.C && y.size(0) == s.N && y.size(3) == s.K, "conv: shape mismatch");
  TORCH_CHECK(s.C % 8 == 0 && s.K % 8 == 0, "conv: channel counts must be padded to multiples of 8");
  TORCH_CHECK(s.P == (s.H + 2 * s.pad - s.R) / s.stride + 1 && s.Q == (s.W + 2 * s.pad - s.S) / s.stride + 1,
              "conv: output size inconsistent with stride/padding");
  TORCH_CHECK(aligned16(x.data_ptr()) && aligned16(w.data_ptr()) && aligned16(y.data_ptr()), "conv: alignment");
  return s;
}

// Split-K workspace of a small-M conv.  The fp32 slabs come fresh from the caching
// allocator (stream ordered, graph-capture safe).  The arrival counters live in a
// persistent per-(device, stream) pool, zeroed ONCE: the in-launch combine resets
// every counter it used before its kernel ends, so launches ordered on one stream
// (and replays of graphs that captured the pool's address) can share it -- a
// per-call at::zeros cost one fill launch per conv (35 fills, ~160 us per step of
// EnhancedCNN at batch 64 on MI355X).  Pools are never freed (a captured graph may
// still point at an outgrown one); they hold a few thousand ints.
struct ConvWs {
  at::Tensor slabs;
  int* cnt = nullptr;
  float* ws() const { return slabs.defined() ? slabs.data_ptr<float>() : nullptr; }
  int* c() const { return cnt; }
};

int* conv_counter_pool(const at::Tensor& like, int64_t n);
// Workspaces of two convs issued in one launch: separate slabs, and counters from one pool
// allocation (the second range after the first).
std::pair<ConvWs, ConvWs> conv_ws2(const ldnn::ConvShape& s0, const ldnn::ConvShape& s1, int op,
                                   const at::Tensor& like);

int* conv_counter_pool(const at::Tensor& like, int64_t n) {
  static std::mutex mu;
  static std::map<std::pair<int, int64_t>, std::vector<at::Tensor>> pools;
  const auto key = std::make_pair((int)like.get_device(), (int64_t)cur_stream(like));
  std::lock_guard<std::mutex> lock(mu);
  auto& v = pools[key];
  if (v.empty() || v.back().numel() < n) {
    const int64_t cap = std::max<int64_t>(n, v.empty() ? 4096 : 2 * v.back().numel());
    v.push_back(at::zeros({cap}, like.options().dtype(at::kInt)));
  }
  return v.back().data_ptr<int>();
}

std::pair<ConvWs, ConvWs> conv_ws2(const ldnn::ConvShape& s0, const ldnn::ConvShape& s1, int op,
                                   const at::Tensor& like) {
  ConvWs w0, w1;
  if (ldnn::get_conv_impl() != 0) return {w0, w1};
  const ldnn::ConvWorkspace n0 = ldnn::conv2d_lds_workspace(s0, op), n1 = ldnn::conv2d_lds_workspace(s1, op);
  if (n0.slab_bytes) w0.slabs = at::empty({(int64_t)(n0.slab_bytes / 4)}, like.options().dtype(at::kFloat));
  if (n1.slab_bytes) w1.slabs = at::empty({(int64_t)(n1.slab_bytes / 4)}, like.options().dtype(at::kFloat));
  if (n0.counters + n1.counters > 0) {
    int* base = conv_counter_pool(like, n0.counters + n1.counters);
    if (n0.counters > 0) w0.cnt = base;
    if (n1.counters > 0) w1.cnt = base + n0.counters;
  }
  return {w0, w1};
}

ConvWs conv_ws(const ldnn::ConvShape& s, int op, const at::Tensor& like) {
  ConvWs w;
  if (ldnn::get_conv_impl() != 0) return w;
  const ldnn::ConvWorkspace need = ldnn::conv2d_lds_workspace(s, op);
  if (need.slab_bytes == 0) return w;
  w.slabs = at::empty({(int64_t)(need.slab_bytes / 4)}, like.options().dtype(at::kFloat));
  if (need.counters > 0) w.cnt = conv_counter_pool(like, need.counters);
  return w;
}

float* fptr_opt(const c10::optional<at::Tensor>& t, int64_t n, const char* name);
const ldnn::BnFin* bn_fwd_fin(ldnn::BnFin& fin, const ldnn::ConvShape& s, const c10::optional<at::Tensor>& bn_ws,
                              const c10::optional<at::Tensor>& bn_gamma, const c10::optional<at::Tensor>& bn_beta,
                              const c10::optional<at::Tensor>& bn_running_mean,
                              const c10::optional<at::Tensor>& bn_running_var,
                              const c10::optional<at::Tensor>& bn_save_mean,
                              const c10::optional<at::Tensor>& bn_save_invstd, double bn_eps, double bn_momentum,
                              const c10::optional<at::Tensor>& bn_num_batches);

// Returns whether the following BatchNorm's statistics were accumulated and
// finalized by the conv epilogue (bn_ws given, LDS-DMA path, no epilogue op).
bool conv_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& y, int64_t stride, int64_t pad,
              const c10::optional<at::Tensor>& bias, int64_t epi, const c10::optional<at::Tensor>& bn_ws,
              const c10::optional<at::Tensor>& bn_gamma, const c10::optional<at::Tensor>& bn_beta,
              const c10::optional<at::Tensor>& bn_running_mean, const c10::optional<at::Tensor>& bn_running_var,
              const c10::optional<at::Tensor>& bn_save_mean, const c10::optional<at::Tensor>& bn_save_invstd,
              double bn_eps, double bn_momentum, const c10::optional<at::Tensor>& bn_num_batches,
              int64_t real_channels, const c10::optional<at::Tensor>& s2d_xs, bool s2d_packed) {
  check_dev(x, at::kBFloat16, "x");
  check_dev(w, at::kBFloat16, "w");
  check_dev(y, at::kBFloat16, "y");
  ldnn::ConvShape s = conv_shape(x, w, y, stride, pad);
  s.c_real = real_channels > 0 && real_channels < s.C ? (int)real_channels : 0;
  uint16_t* xs = nullptr;
  if (s2d_xs.has_value()) {
    check_dev(*s2d_xs, at::kBFloat16, "s2d_xs");
    TORCH_CHECK(ldnn::stem_s2d_fwd_ok(s), "conv_fwd: s2d_xs given for a shape the s2d stem forward does not take");
    TORCH_CHECK(s2d_xs->is_contiguous() && s2d_xs->dim() == 4 && s2d_xs->size(0) == s.N && s2d_xs->size(1) == s.P + 3 &&
                    s2d_xs->size(2) == s.Q + 3 && s2d_xs->size(3) == 16,
                "conv_fwd: s2d_xs must be a dense [N][P+3][Q+3][16] bf16 tensor");
    xs = bf16_mut(*s2d_xs);
    s.s2d_packed = s2d_packed ? 1 : 0;
  }
  TORCH_CHECK(!s2d_packed || s2d_xs.has_value(), "conv_fwd: s2d_packed needs s2d_xs");
  const float* b = nullptr;
  if (bias.has_value()) {
    check_dev(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() >= s.K && aligned16(bias->data_ptr()), "conv: bad bias");
    b = bias->data_ptr<float>();
  }
  TORCH_CHECK(epi == ldnn::EPI_NONE || b != nullptr, "conv: bias epilogue needs a bias");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  const ConvWs ws = conv_ws(s, 0, x);
  ldnn::BnFin fin{};
  TORCH_CHECK(!bn_ws.has_value() || epi == ldnn::EPI_NONE, "conv: fused BN statistics need a plain (EPI_NONE) conv");
  const ldnn::BnFin* finp = bn_fwd_fin(fin, s, bn_ws, bn_gamma, bn_beta, bn_running_mean, bn_running_var, bn_save_mean,
                                       bn_save_invstd, bn_eps, bn_momentum, bn_num_batches);
  bool done = false;
  check(ldnn::conv2d_fwd(s, bf16_ptr(x), bf16_ptr(w), bf16_mut(y), b, (int)epi, cur_stream(x), ws.ws(), ws.c(),
                         finp, &done, xs),
        "conv2d_fwd");
  return done;
}

// The fused next-BN statistics state of a forward conv (nullptr without bn_ws).
const ldnn::BnFin* bn_fwd_fin(ldnn::BnFin& fin, const ldnn::ConvShape& s, const c10::optional<at::Tensor>& bn_ws,
                              const c10::optional<at::Tensor>& bn_gamma, const c10::optional<at::Tensor>& bn_beta,
                              const c10::optional<at::Tensor>& bn_running_mean,
                              const c10::optional<at::Tensor>& bn_running_var,
                              const c10::optional<at::Tensor>& bn_save_mean,
                              const c10::optional<at::Tensor>& bn_save_invstd, double bn_eps, double bn_momentum,
                              const c10::optional<at::Tensor>& bn_num_batches) {
  const ldnn::BnFin* finp = nullptr;
  if (bn_ws.has_value()) {
    const int C = s.K;
    ldnn::BnArgs a{};
    a.M = s.N * s.P * s.Q;
    a.C = C;
    a.gamma = fptr_opt(bn_gamma, C, "bn_gamma");
    a.beta = fptr_opt(bn_beta, C, "bn_beta");
    a.running_mean = fptr_opt(bn_running_mean, C, "bn_running_mean");
    a.running_var = fptr_opt(bn_running_var, C, "bn_running_var");
    a.save_mean = fptr_opt(bn_save_mean, C, "bn_save_mean");
    a.save_invstd = fptr_opt(bn_save_invstd, C, "bn_save_invstd");
    TORCH_CHECK(a.save_mean && a.save_invstd, "conv: fused BN statistics need save_mean / save_invstd");
    a.ws = fptr_opt(bn_ws, ldnn::bn_workspace_floats(C), "bn_ws");
    a.eps = (float)bn_eps;
    a.momentum = (float)bn_momentum;
    if (bn_num_batches.has_value()) {
      check_dev(*bn_num_batches, at::kLong, "bn_num_batches");
      a.num_batches = bn_num_batches->data_ptr<int64_t>();
    }
    fin = ldnn::bn_forward_fin_conv(a);
    finp = &fin;
  }
  return finp;
}

c10::optional<at::Tensor> opt_item(const py::dict& d, const char* k) {
  if (!d.contains(k) || d[k].is_none()) return c10::nullopt;
  return d[k].cast<at::Tensor>();
}
const ldnn::BnFin* bn_fwd_fin_dict(ldnn::BnFin& fin, const ldnn::ConvShape& s, const py::object& bn) {
  if (bn.is_none()) return nullptr;
  const py::dict d = bn.cast<py::dict>();
  const double eps = d.contains("eps") ? d["eps"].cast<double>() : 1e-5;
  const double mom = d.contains("momentum") ? d["momentum"].cast<double>() : 0.1;
  return bn_fwd_fin(fin, s, opt_item(d, "ws"), opt_item(d, "gamma"), opt_item(d, "beta"), opt_item(d, "running_mean"),
                    opt_item(d, "running_var"), opt_item(d, "save_mean"), opt_item(d, "save_invstd"), eps, mom,
                    opt_item(d, "num_batches"));
}

// A downsampling block's 3x3 conv (w0 -> y0) and 1x1 shortcut conv (w1 -> y1) of one input x,
// each with its next BN's fused statistics (bn0 / bn1: None or a dict of conv_fwd's bn_*
// arguments without the prefix): one launch where the kernels allow.  Returns the two flags.
std::tuple<bool, bool> conv_fwd2(const at::Tensor& x, const at::Tensor& w0, const at::Tensor& y0, int64_t stride0,
                                 int64_t pad0, const at::Tensor& w1, const at::Tensor& y1, int64_t stride1,
                                 int64_t pad1, const py::object& bn0, const py::object& bn1) {
  check_dev(x, at::kBFloat16, "x");
  check_dev(w0, at::kBFloat16, "w0");
  check_dev(y0, at::kBFloat16, "y0");
  check_dev(w1, at::kBFloat16, "w1");
  check_dev(y1, at::kBFloat16, "y1");
  const ldnn::ConvShape s0 = conv_shape(x, w0, y0, stride0, pad0);
  const ldnn::ConvShape s1 = conv_shape(x, w1, y1, stride1, pad1);
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  const ConvWs ws0 = conv_ws(s0, 0, x);
  const ConvWs ws1 = conv_ws(s1, 0, x);
  ldnn::BnFin f0{}, f1{};
  const ldnn::BnFin* p0 = bn_fwd_fin_dict(f0, s0, bn0);
  const ldnn::BnFin* p1 = bn_fwd_fin_dict(f1, s1, bn1);
  bool d0 = false, d1 = false;
  check(ldnn::conv2d_fwd2(s0, bf16_ptr(x), bf16_ptr(w0), bf16_mut(y0), ws0.ws(), ws0.c(), p0, &d0, s1, bf16_ptr(w1),
                          bf16_mut(y1), ws1.ws(), ws1.c(), p1, &d1, cur_stream(x)),
        "conv2d_fwd2");
  return {d0, d1};
}

// bn_x given: dx is the gradient of a training BatchNorm(+ReLU)'s output (bn_x = that BN's
// input, bn_mask its ReLU bits); returns whether the dgrad's epilogue also accumulated and
// finalized that BN's backward statistics (then bn_bwd(..., stats_ready=True) applies them).
// The BnBwdFuse of conv_dgrad / conv_bwd's optional BN arguments (nullptr without bn_x).
const ldnn::BnBwdFuse* bn_bwd_fuse(ldnn::BnBwdFuse& fuse, const ldnn::ConvShape& s,
                                   const c10::optional<at::Tensor>& bn_x, const c10::optional<at::Tensor>& bn_mask,
                                   const c10::optional<at::Tensor>& bn_ws, const c10::optional<at::Tensor>& bn_gamma,
                                   const c10::optional<at::Tensor>& bn_save_mean,
                                   const c10::optional<at::Tensor>& bn_save_invstd,
                                   const c10::optional<at::Tensor>& bn_dgamma,
                                   const c10::optional<at::Tensor>& bn_dbeta, bool bn_assign) {
  const ldnn::BnBwdFuse* fp = nullptr;
  if (bn_x.has_value()) {
    const int C = s.C;
    const int64_t M = (int64_t)s.N * s.H * s.W;
    check_dev(*bn_x, at::kBFloat16, "bn_x");
    TORCH_CHECK(bn_x->is_contiguous() && bn_x->numel() == M * C, "conv_dgrad: bn_x must be dense [M][C] like dx");
    ldnn::BnArgs a{};
    a.M = (int)M;
    a.C = C;
    a.gamma = fptr_opt(bn_gamma, C, "bn_gamma");
    a.save_mean = fptr_opt(bn_save_mean, C, "bn_save_mean");
    a.save_invstd = fptr_opt(bn_save_invstd, C, "bn_save_invstd");
    TORCH_CHECK(a.save_mean && a.save_invstd, "conv_dgrad: the BN statistics need save_mean / save_invstd");
    a.ws = fptr_opt(bn_ws, ldnn::bn_workspace_floats(C), "bn_ws");
    TORCH_CHECK(a.ws != nullptr, "conv_dgrad: bn_ws");
    fuse.fin = ldnn::bn_backward_fin_conv(a, fptr_opt(bn_dgamma, C, "bn_dgamma"), fptr_opt(bn_dbeta, C, "bn_dbeta"),
                                          bn_assign);
    fuse.x = bf16_ptr(*bn_x);
    if (bn_mask.has_value()) {
      check_dev(*bn_mask, at::kByte, "bn_mask");
      TORCH_CHECK(bn_mask->is_contiguous() && bn_mask->numel() == M * C / 8, "conv_dgrad: bn_mask [M][C/8]");
      fuse.mask = bn_mask->data_ptr<uint8_t>();
    }
    fp = &fuse;
  }
  return fp;
}

bool conv_dgrad(const at::Tensor& dy, const at::Tensor& w, const at::Tensor& dx, int64_t stride, int64_t pad,
                const c10::optional<at::Tensor>& bn_x, const c10::optional<at::Tensor>& bn_mask,
                const c10::optional<at::Tensor>& bn_ws, const c10::optional<at::Tensor>& bn_gamma,
                const c10::optional<at::Tensor>& bn_save_mean, const c10::optional<at::Tensor>& bn_save_invstd,
                const c10::optional<at::Tensor>& bn_dgamma, const c10::optional<at::Tensor>& bn_dbeta,
                bool bn_assign) {
  check_dev(dy, at::kBFloat16, "dy");
  check_dev(w, at::kBFloat16, "w");
  check_dev(dx, at::kBFloat16, "dx");
  ldnn::ConvShape s = conv_shape(dx, w, dy, stride, pad);
  c10::hip::HIPGuardMasqueradingAsCUDA g(dy.device());
  const ConvWs ws = conv_ws(s, 1, dy);
  ldnn::BnBwdFuse fuse{};
  const ldnn::BnBwdFuse* fp = bn_bwd_fuse(fuse, s, bn_x, bn_mask, bn_ws, bn_gamma, bn_save_mean, bn_save_invstd,
                                          bn_dgamma, bn_dbeta, bn_assign);
  bool done = false;
  check(ldnn::conv2d_dgrad(s, bf16_ptr(dy), bf16_ptr(w), bf16_mut(dx), cur_stream(dy), ws.ws(), ws.c(), fp, &done),
        "conv2d_dgrad");
  return done;
}

ldnn::ConvShape wgrad_shape(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& dw, int64_t stride,
                            int64_t pad, int64_t real_channels) {
  TORCH_CHECK(dw.dim() == 4 && dw.is_contiguous(), "conv_wgrad: dw must be a dense [K][R][S][C] fp32 tensor");
  ldnn::ConvShape s{};
  TORCH_CHECK(x.dim() == 4 && dy.dim() == 4 && x.is_contiguous() && dy.is_contiguous(), "conv_wgrad: layout");
  s.N = (int)x.size(0); s.H = (int)x.size(1); s.W = (int)x.size(2); s.C = (int)x.size(3);
  s.K = (int)dw.size(0); s.R = (int)dw.size(1); s.S = (int)dw.size(2);
  s.P = (int)dy.size(1); s.Q = (int)dy.size(2);
  s.stride = (int)stride; s.pad = (int)pad;
  s.c_real = real_channels > 0 && real_channels < s.C ? (int)real_channels : 0;
  TORCH_CHECK(dw.size(3) == s.C && dy.size(3) == s.K && dy.size(0) == s.N, "conv_wgrad: shape mismatch");
  TORCH_CHECK(s.C % 8 == 0 && s.K % 8 == 0, "conv_wgrad: channels must be multiples of 8");
  return s;
}

// A downsampling block's two convs of one input x, backward: (dy_k, w_k -> dx_k; dy_k, x -> dw_k
// with beta_k) for k = 0, 1 -- both dgrads and wgrads in one launch where the kernels allow.
void conv_bwd2(const at::Tensor& x, const at::Tensor& dy0, const at::Tensor& w0, const at::Tensor& dx0,
               const at::Tensor& dw0, int64_t stride0, int64_t pad0, double beta0, const at::Tensor& dy1,
               const at::Tensor& w1, const at::Tensor& dx1, const at::Tensor& dw1, int64_t stride1, int64_t pad1,
               double beta1, int64_t real_channels) {
  check_dev(x, at::kBFloat16, "x");
  ldnn::BwdJob j[2];
  const at::Tensor* dys[2] = {&dy0, &dy1};
  const at::Tensor* ws[2] = {&w0, &w1};
  const at::Tensor* dxs[2] = {&dx0, &dx1};
  const at::Tensor* dws[2] = {&dw0, &dw1};
  const int64_t strides[2] = {stride0, stride1}, pads[2] = {pad0, pad1};
  const double betas[2] = {beta0, beta1};
  for (int c = 0; c < 2; ++c) {
    check_dev(*dys[c], at::kBFloat16, "dy");
    check_dev(*ws[c], at::kBFloat16, "w");
    check_dev(*dxs[c], at::kBFloat16, "dx");
    check_dev(*dws[c], at::kFloat, "dw");
    TORCH_CHECK(dxs[c]->sizes() == x.sizes(), "conv_bwd2: dx must have x's shape");
    j[c].sd = conv_shape(*dxs[c], *ws[c], *dys[c], strides[c], pads[c]);
    j[c].sw = wgrad_shape(*dys[c], x, *dws[c], strides[c], pads[c], real_channels);
    j[c].dy = bf16_ptr(*dys[c]);
    j[c].w = bf16_ptr(*ws[c]);
    j[c].dx = bf16_mut(*dxs[c]);
    j[c].dw = dws[c]->data_ptr<float>();
    j[c].beta = (float)betas[c];
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  const auto wd = conv_ws2(j[0].sd, j[1].sd, 1, x);
  const auto ww = conv_ws2(j[0].sw, j[1].sw, 2, x);
  j[0].ws_d = wd.first.ws();
  j[0].cnt_d = wd.first.c();
  j[1].ws_d = wd.second.ws();
  j[1].cnt_d = wd.second.c();
  j[0].ws_w = ww.first.ws();
  j[1].ws_w = ww.second.ws();
  check(ldnn::conv2d_bwd2(j[0], j[1], bf16_ptr(x), cur_stream(x)), "conv2d_bwd2");
}

// A conv layer's backward: dx (conv_dgrad, optional BN statistics) AND dw (conv_wgrad, beta /
// real_channels) from one dy -- one launch for both where the kernels allow (conv2d_bwd).
bool conv_bwd(const at::Tensor& dy, const at::Tensor& w, const at::Tensor& dx, const at::Tensor& x,
              const at::Tensor& dw, int64_t stride, int64_t pad, double beta, int64_t real_channels,
              const c10::optional<at::Tensor>& bn_x, const c10::optional<at::Tensor>& bn_mask,
              const c10::optional<at::Tensor>& bn_ws, const c10::optional<at::Tensor>& bn_gamma,
              const c10::optional<at::Tensor>& bn_save_mean, const c10::optional<at::Tensor>& bn_save_invstd,
              const c10::optional<at::Tensor>& bn_dgamma, const c10::optional<at::Tensor>& bn_dbeta,
              bool bn_assign) {
  check_dev(dy, at::kBFloat16, "dy");
  check_dev(w, at::kBFloat16, "w");
  check_dev(dx, at::kBFloat16, "dx");
  check_dev(x, at::kBFloat16, "x");
  check_dev(dw, at::kFloat, "dw");
  const ldnn::ConvShape sd = conv_shape(dx, w, dy, stride, pad);
  const ldnn::ConvShape sw = wgrad_shape(dy, x, dw, stride, pad, real_channels);
  c10::hip::HIPGuardMasqueradingAsCUDA g(dy.device());
  const ConvWs wsd = conv_ws(sd, 1, dy);
  const ConvWs wsw = conv_ws(sw, 2, dy);
  ldnn::BnBwdFuse fuse{};
  const ldnn::BnBwdFuse* fp = bn_bwd_fuse(fuse, sd, bn_x, bn_mask, bn_ws, bn_gamma, bn_save_mean, bn_save_invstd,
                                          bn_dgamma, bn_dbeta, bn_assign);
  bool done = false;
  check(ldnn::conv2d_bwd(sd, bf16_ptr(dy), bf16_ptr(w), bf16_mut(dx), wsd.ws(), wsd.c(), fp, &done, sw, bf16_ptr(x),
                         dw.data_ptr<float>(), (float)beta, wsw.ws(), cur_stream(dy)),
        "conv2d_bwd");
  return done;
}

void conv_wgrad(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& dw, int64_t stride, int64_t pad,
                double beta, int64_t real_channels, const c10::optional<at::Tensor>& s2d_xs) {
  check_dev(dy, at::kBFloat16, "dy");
  check_dev(x, at::kBFloat16, "x");
  check_dev(dw, at::kFloat, "dw");
  const ldnn::ConvShape s = wgrad_shape(dy, x, dw, stride, pad, real_channels);
  const uint16_t* xs = nullptr;
  if (s2d_xs.has_value()) {
    check_dev(*s2d_xs, at::kBFloat16, "s2d_xs");
    TORCH_CHECK(ldnn::stem_s2d_fwd_ok(s) && s2d_xs->is_contiguous() && s2d_xs->numel() == (int64_t)s.N * (s.P + 3) * (s.Q + 3) * 16,
                "conv_wgrad: s2d_xs must be the forward's packed [N][P+3][Q+3][16] image");
    xs = bf16_ptr(*s2d_xs);
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(dy.device());
  const ConvWs ws = conv_ws(s, 2, dy);
  check(ldnn::conv2d_wgrad(s, bf16_ptr(dy), bf16_ptr(x), dw.data_ptr<float>(), (float)beta, cur_stream(dy), ws.ws(),
                           xs),
        "conv2d_wgrad");
}

float* fptr_opt(const c10::optional<at::Tensor>& t, int64_t n, const char* name) {
  if (!t.has_value()) return nullptr;
  check_dev(*t, at::kFloat, name);
  TORCH_CHECK(t->is_contiguous() && t->numel() >= n, name, ": bad tensor");
  return t->data_ptr<float>();
}

// x, y, residual: dense [M][C] bf16 (NHWC flattened); stats: [C] fp32; ws: fp32 [4C + 2C]
void bn_fwd(const at::Tensor& x, const at::Tensor& y, const c10::optional<at::Tensor>& residual,
            const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& beta,
            const c10::optional<at::Tensor>& running_mean, const c10::optional<at::Tensor>& running_var,
            const at::Tensor& save_mean, const at::Tensor& save_invstd, const at::Tensor& ws, double eps,
            double momentum, bool training, bool relu, const c10::optional<at::Tensor>& num_batches,
            bool stats_ready, const c10::optional<at::Tensor>& mask) {
  check_dev(x, at::kBFloat16, "x");
  check_dev(y, at::kBFloat16, "y");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && y.sizes() == x.sizes() && y.is_contiguous(), "bn: [M][C] dense");
  const int64_t M = x.size(0), C = x.size(1);
  TORCH_CHECK(C % 8 == 0, "bn: C must be a multiple of 8");
  ldnn::BnArgs a{};
  a.x = bf16_ptr(x);
  a.y = bf16_mut(y);
  if (residual.has_value()) {
    check_dev(*residual, at::kBFloat16, "residual");
    TORCH_CHECK(residual->sizes() == x.sizes() && residual->is_contiguous(), "bn: residual layout");
    a.residual = bf16_ptr(*residual);
  }
  a.gamma = fptr_opt(gamma, C, "gamma");
  a.beta = fptr_opt(beta, C, "beta");
  a.running_mean = fptr_opt(running_mean, C, "running_mean");
  a.running_var = fptr_opt(running_var, C, "running_var");
  a.save_mean = fptr_opt(save_mean, C, "save_mean");
  a.save_invstd = fptr_opt(save_invstd, C, "save_invstd");
  a.ws = fptr_opt(ws, ldnn::bn_workspace_floats((int)C), "ws");
  a.M = (int)M;
  a.C = (int)C;
  a.eps = (float)eps;
  a.momentum = (float)momentum;
  a.training = training ? 1 : 0;
  a.relu = relu ? 1 : 0;
  TORCH_CHECK(training || (a.running_mean && a.running_var), "bn: eval mode needs running statistics");
  if (mask.has_value()) {  // ReLU bit mask [M][C/8] for the backward
    check_dev(*mask, at::kByte, "mask");
    TORCH_CHECK(relu && mask->is_contiguous() && mask->numel() == M * C / 8, "bn: mask needs relu and [M][C/8] bytes");
    a.mask = mask->data_ptr<uint8_t>();
  }
  if (num_batches.has_value() && training) {
    check_dev(*num_batches, at::kLong, "num_batches");
    a.num_batches = num_batches->data_ptr<int64_t>();
  }
  if (stats_ready) {  // the producing conv's epilogue already finalized scale / shift into ws
    TORCH_CHECK(training, "bn: stats_ready is a training-mode path");
    check(ldnn::bn_forward_apply(a, cur_stream(x)), "bn_forward_apply");
    return;
  }
  check(ldnn::bn_forward(a, cur_stream(x)), "bn_forward");
}

void bn_bwd(const at::Tensor& x, const at::Tensor& y, const at::Tensor& dy, const at::Tensor& dx,
            const c10::optional<at::Tensor>& dres, const c10::optional<at::Tensor>& gamma,
            const at::Tensor& save_mean, const at::Tensor& save_invstd, const at::Tensor& ws,
            const c10::optional<at::Tensor>& dgamma, const c10::optional<at::Tensor>& dbeta, bool relu,
            const c10::optional<at::Tensor>& mask, bool grad_assign, const c10::optional<at::Tensor>& dy2,
            bool stats_ready) {
  check_dev(x, at::kBFloat16, "x");
  check_dev(dy, at::kBFloat16, "dy");
  check_dev(dx, at::kBFloat16, "dx");
  TORCH_CHECK(!(stats_ready && dy2.has_value()), "bn_bwd: stats_ready covers dy alone");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && dy.sizes() == x.sizes() && dy.is_contiguous() &&
                  dx.sizes() == x.sizes() && dx.is_contiguous(),
              "bn_bwd: [M][C] dense tensors");
  const int64_t M = x.size(0), C = x.size(1);
  ldnn::BnArgs a{};
  a.x = bf16_ptr(x);
  a.y = bf16_mut(y);
  a.gamma = fptr_opt(gamma, C, "gamma");
  a.save_mean = fptr_opt(save_mean, C, "save_mean");
  a.save_invstd = fptr_opt(save_invstd, C, "save_invstd");
  a.ws = fptr_opt(ws, ldnn::bn_workspace_floats((int)C), "ws");
  a.M = (int)M;
  a.C = (int)C;
  a.relu = relu ? 1 : 0;
  if (mask.has_value()) {  // relu'(y) from the forward's bit mask instead of y
    check_dev(*mask, at::kByte, "mask");
    TORCH_CHECK(relu && mask->is_contiguous() && mask->numel() == M * C / 8, "bn_bwd: mask needs relu, [M][C/8]");
    a.mask = mask->data_ptr<uint8_t>();
  }
  if (dy2.has_value()) {
    check_dev(*dy2, at::kBFloat16, "dy2");
    TORCH_CHECK(dy2->sizes() == x.sizes() && dy2->is_contiguous(), "bn_bwd: dy2 layout");
    a.dy2 = bf16_ptr(*dy2);
  }
  uint16_t* dr = nullptr;
  if (dres.has_value()) {
    check_dev(*dres, at::kBFloat16, "dres");
    TORCH_CHECK(dres->sizes() == x.sizes() && dres->is_contiguous(), "bn_bwd: dres layout");
    dr = bf16_mut(*dres);
  }
  check(ldnn::bn_backward(a, bf16_ptr(dy), bf16_mut(dx), dr, fptr_opt(dgamma, C, "dgamma"),
                          fptr_opt(dbeta, C, "dbeta"), cur_stream(x), grad_assign, stats_ready),
        "bn_backward");
}

// x [N][H][W][C], y [N][P][Q][C] dense bf16; argmax uint8 [N][P][Q][C] for max pooling
void pool_fwd(const at::Tensor& x, const at::Tensor& y, const c10::optional<at::Tensor>& argmax, int64_t R,
              int64_t S, int64_t stride, int64_t pad, bool is_max, bool nchw_out) {
  check_dev(x, at::kBFloat16, "x");
  check_dev(y, at::kBFloat16, "y");
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && x.is_contiguous() && y.is_contiguous(), "pool: dense NHWC");
  // nchw_out: y is [N][Cl][P][Q] (Cl <= C logical channels), argmax keeps the NHWC [N][P][Q][C] layout
  const int64_t P = nchw_out ? y.size(2) : y.size(1), Q = nchw_out ? y.size(3) : y.size(2);
  const int64_t cl = nchw_out ? y.size(1) : 0;
  TORCH_CHECK(y.size(0) == x.size(0) && (nchw_out ? cl <= x.size(3) : y.size(3) == x.size(3)), "pool: y shape");
  uint8_t* am = nullptr;
  if (is_max) {
    TORCH_CHECK(argmax.has_value() && argmax->scalar_type() == at::kByte &&
                    argmax->numel() == x.size(0) * P * Q * x.size(3),
                "pool: max pooling needs a uint8 argmax tensor");
    am = argmax->data_ptr<uint8_t>();
    TORCH_CHECK(argmax->is_contiguous() && ((uintptr_t)am & 7) == 0, "pool: argmax must be dense and 8-B aligned");
  }
  check(ldnn::pool2d_fwd(bf16_ptr(x), bf16_mut(y), am, (int)x.size(0), (int)x.size(1), (int)x.size(2),
                         (int)x.size(3), (int)P, (int)Q, (int)R, (int)S, (int)stride, (int)pad, is_max,
                         cur_stream(x), (int)cl),
        "pool2d_fwd");
}

void pool_bwd(const at::Tensor& dy, const c10::optional<at::Tensor>& argmax, const at::Tensor& dx, int64_t R,
              int64_t S, int64_t stride, int64_t pad, bool is_max, const c10::optional<at::Tensor>& dy2,
              bool nchw_dy) {
  check_dev(dy, at::kBFloat16, "dy");
  check_dev(dx, at::kBFloat16, "dx");
  TORCH_CHECK(dy.dim() == 4 && dx.dim() == 4 && dy.is_contiguous() && dx.is_contiguous(), "pool_bwd: dense NHWC");
  // nchw_dy: dy is [N][Cl][P][Q] (the NCHW output of pool_fwd(nchw_out=True))
  const int64_t P = nchw_dy ? dy.size(2) : dy.size(1), Q = nchw_dy ? dy.size(3) : dy.size(2);
  const int64_t cl = nchw_dy ? dy.size(1) : 0;
  TORCH_CHECK(dy.size(0) == dx.size(0) && (nchw_dy ? cl <= dx.size(3) : dy.size(3) == dx.size(3)),
              "pool_bwd: dy shape");
  TORCH_CHECK(!(nchw_dy && dy2.has_value()), "pool_bwd: dy2 needs the NHWC gradient");
  const uint8_t* am = nullptr;
  if (is_max) {
    TORCH_CHECK(argmax.has_value() && argmax->numel() == dx.size(0) * P * Q * dx.size(3), "pool_bwd: argmax");
    am = argmax->data_ptr<uint8_t>();
    TORCH_CHECK(argmax->is_contiguous() && ((uintptr_t)am & 7) == 0, "pool: argmax must be dense and 8-B aligned");
  }
  const uint16_t* d2 = nullptr;
  if (dy2.has_value()) {
    check_dev(*dy2, at::kBFloat16, "dy2");
    TORCH_CHECK(dy2->sizes() == dy.sizes() && dy2->is_contiguous(), "pool_bwd: dy2 layout");
    d2 = bf16_ptr(*dy2);
  }
  check(ldnn::pool2d_bwd(bf16_ptr(dy), am, bf16_mut(dx), (int)dx.size(0), (int)dx.size(1), (int)dx.size(2),
                         (int)dx.size(3), (int)P, (int)Q, (int)R, (int)S, (int)stride, (int)pad,
                         is_max, cur_stream(dy), d2, (int)cl),
        "pool2d_bwd");
}

// y = relu(bn_a(x) + bn_b(r)): residual block tail whose shortcut carries its own BatchNorm
// (the shortcut BN's output is never stored).  x, r, y: [M][C] dense bf16.
ldnn::BnArgs dual_args(const at::Tensor& x, const c10::optional<at::Tensor>& gamma,
                       const c10::optional<at::Tensor>& beta, const c10::optional<at::Tensor>& running_mean,
                       const c10::optional<at::Tensor>& running_var, const at::Tensor& save_mean,
                       const at::Tensor& save_invstd, const at::Tensor& ws, double eps, double momentum,
                       const c10::optional<at::Tensor>& num_batches) {
  const int64_t M = x.size(0), C = x.size(1);
  ldnn::BnArgs a{};
  a.x = bf16_ptr(x);
  a.gamma = fptr_opt(gamma, C, "gamma");
  a.beta = fptr_opt(beta, C, "beta");
  a.running_mean = fptr_opt(running_mean, C, "running_mean");
  a.running_var = fptr_opt(running_var, C, "running_var");
  a.save_mean = fptr_opt(save_mean, C, "save_mean");
  a.save_invstd = fptr_opt(save_invstd, C, "save_invstd");
  a.ws = fptr_opt(ws, ldnn::bn_workspace_floats((int)C), "ws");
  a.M = (int)M;
  a.C = (int)C;
  a.eps = (float)eps;
  a.momentum = (float)momentum;
  a.training = 1;
  if (num_batches.has_value()) {
    check_dev(*num_batches, at::kLong, "num_batches");
    a.num_batches = num_batches->data_ptr<int64_t>();
  }
  return a;
}

void bn_dual_fwd(const at::Tensor& x, const at::Tensor& r, const at::Tensor& y, const c10::optional<at::Tensor>& mask,
                 const c10::optional<at::Tensor>& gamma_a, const c10::optional<at::Tensor>& beta_a,
                 const c10::optional<at::Tensor>& rm_a, const c10::optional<at::Tensor>& rv_a,
                 const at::Tensor& mean_a, const at::Tensor& invstd_a, const at::Tensor& ws_a, double eps_a,
                 double mom_a, const c10::optional<at::Tensor>& nb_a, bool ready_a,
                 const c10::optional<at::Tensor>& gamma_b, const c10::optional<at::Tensor>& beta_b,
                 const c10::optional<at::Tensor>& rm_b, const c10::optional<at::Tensor>& rv_b,
                 const at::Tensor& mean_b, const at::Tensor& invstd_b, const at::Tensor& ws_b, double eps_b,
                 double mom_b, const c10::optional<at::Tensor>& nb_b, bool ready_b) {
  for (const at::Tensor* t : {&x, &r, &y}) {
    check_dev(*t, at::kBFloat16, "bn_dual_fwd tensor");
    TORCH_CHECK(t->dim() == 2 && t->is_contiguous() && t->sizes() == x.sizes(), "bn_dual_fwd: [M][C] dense");
  }
  TORCH_CHECK(x.size(1) % 8 == 0, "bn_dual_fwd: C % 8");
  ldnn::BnArgs a = dual_args(x, gamma_a, beta_a, rm_a, rv_a, mean_a, invstd_a, ws_a, eps_a, mom_a, nb_a);
  ldnn::BnArgs b = dual_args(r, gamma_b, beta_b, rm_b, rv_b, mean_b, invstd_b, ws_b, eps_b, mom_b, nb_b);
  a.y = bf16_mut(y);
  a.relu = 1;
  if (mask.has_value()) {
    check_dev(*mask, at::kByte, "mask");
    TORCH_CHECK(mask->is_contiguous() && mask->numel() == x.numel() / 8, "bn_dual_fwd: mask [M][C/8]");
    a.mask = mask->data_ptr<uint8_t>();
  }
  check(ldnn::bn_dual_forward(a, b, ready_a, ready_b, cur_stream(x)), "bn_dual_forward");
}

void bn_dual_bwd(const at::Tensor& x, const at::Tensor& r, const at::Tensor& y, const c10::optional<at::Tensor>& mask,
                 const at::Tensor& dy, const c10::optional<at::Tensor>& dy2, const at::Tensor& dx,
                 const at::Tensor& dr, const c10::optional<at::Tensor>& gamma_a, const at::Tensor& mean_a,
                 const at::Tensor& invstd_a, const at::Tensor& ws_a, const c10::optional<at::Tensor>& dgamma_a,
                 const c10::optional<at::Tensor>& dbeta_a, bool assign_a, const c10::optional<at::Tensor>& gamma_b,
                 const at::Tensor& mean_b, const at::Tensor& invstd_b, const at::Tensor& ws_b,
                 const c10::optional<at::Tensor>& dgamma_b, const c10::optional<at::Tensor>& dbeta_b,
                 bool assign_b) {
  for (const at::Tensor* t : {&x, &r, &dy, &dx, &dr}) {
    check_dev(*t, at::kBFloat16, "bn_dual_bwd tensor");
    TORCH_CHECK(t->dim() == 2 && t->is_contiguous() && t->sizes() == x.sizes(), "bn_dual_bwd: [M][C] dense");
  }
  const int64_t C = x.size(1);
  ldnn::BnArgs a = dual_args(x, gamma_a, c10::nullopt, c10::nullopt, c10::nullopt, mean_a, invstd_a, ws_a, 0.0, 0.0,
                             c10::nullopt);
  ldnn::BnArgs b = dual_args(r, gamma_b, c10::nullopt, c10::nullopt, c10::nullopt, mean_b, invstd_b, ws_b, 0.0, 0.0,
                             c10::nullopt);
  a.relu = 1;
  if (mask.has_value()) {
    check_dev(*mask, at::kByte, "mask");
    TORCH_CHECK(mask->is_contiguous() && mask->numel() == x.numel() / 8, "bn_dual_bwd: mask [M][C/8]");
    a.mask = mask->data_ptr<uint8_t>();
  } else {
    check_dev(y, at::kBFloat16, "y");
    TORCH_CHECK(y.sizes() == x.sizes() && y.is_contiguous(), "bn_dual_bwd: y layout");
    a.y = bf16_mut(y);
  }
  if (dy2.has_value()) {
    check_dev(*dy2, at::kBFloat16, "dy2");
    TORCH_CHECK(dy2->sizes() == x.sizes() && dy2->is_contiguous(), "bn_dual_bwd: dy2 layout");
    a.dy2 = bf16_ptr(*dy2);
  }
  check(ldnn::bn_dual_backward(a, b, bf16_ptr(dy), bf16_mut(dx), bf16_mut(dr), fptr_opt(dgamma_a, C, "dgamma_a"),
                               fptr_opt(dbeta_a, C, "dbeta_a"), fptr_opt(dgamma_b, C, "dgamma_b"),
                               fptr_opt(dbeta_b, C, "dbeta_b"), assign_a, assign_b, cur_stream(x)),
        "bn_dual_backward");
}

// relu(BN(x)) -> 3x3/2 max-pool in one pass: x [N][H][W][C] (pre-BN), y / argmax [N][P][Q][C]
bool bn_pool_fwd(const at::Tensor& x, const at::Tensor& y, const at::Tensor& argmax,
                 const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& beta,
                 const c10::optional<at::Tensor>& running_mean, const c10::optional<at::Tensor>& running_var,
                 const at::Tensor& save_mean, const at::Tensor& save_invstd, const at::Tensor& ws, double eps,
                 double momentum, const c10::optional<at::Tensor>& num_batches, bool stats_ready, int64_t pad,
                 const c10::optional<at::Tensor>& xam) {
  check_dev(x, at::kBFloat16, "x");
  check_dev(y, at::kBFloat16, "y");
  check_dev(argmax, at::kByte, "argmax");
  uint16_t* xam_p = nullptr;
  if (xam.has_value()) {
    check_dev(*xam, at::kBFloat16, "xam");
    TORCH_CHECK(xam->sizes() == y.sizes() && xam->is_contiguous(), "bn_pool_fwd: xam must be laid out as y");
    xam_p = bf16_mut(*xam);
  }
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && x.is_contiguous() && y.is_contiguous() && argmax.is_contiguous() &&
                  argmax.sizes() == y.sizes() && y.size(0) == x.size(0) && y.size(3) == x.size(3),
              "bn_pool_fwd: dense NHWC x / y / argmax");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  ldnn::BnArgs a{};
  a.x = bf16_ptr(x);
  a.gamma = fptr_opt(gamma, C, "gamma");
  a.beta = fptr_opt(beta, C, "beta");
  a.running_mean = fptr_opt(running_mean, C, "running_mean");
  a.running_var = fptr_opt(running_var, C, "running_var");
  a.save_mean = fptr_opt(save_mean, C, "save_mean");
  a.save_invstd = fptr_opt(save_invstd, C, "save_invstd");
  a.ws = fptr_opt(ws, ldnn::bn_workspace_floats((int)C), "ws");
  a.M = (int)(N * H * W);
  a.C = (int)C;
  a.eps = (float)eps;
  a.momentum = (float)momentum;
  a.training = 1;
  a.relu = 1;
  if (num_batches.has_value()) {
    check_dev(*num_batches, at::kLong, "num_batches");
    a.num_batches = num_batches->data_ptr<int64_t>();
  }
  uint8_t* am = argmax.data_ptr<uint8_t>();
  TORCH_CHECK(((uintptr_t)am & 7) == 0, "bn_pool_fwd: argmax must be 8-B aligned");
  check(ldnn::bn_maxpool_forward(a, (int)N, (int)H, (int)W, (int)y.size(1), (int)y.size(2), (int)pad, bf16_mut(y),
                                 am, stats_ready, cur_stream(x), xam_p),
        "bn_maxpool_forward (3x3/2 window, C/8 dividing 256)");
  return true;
}

void bn_pool_bwd(const at::Tensor& x, const at::Tensor& dy, const at::Tensor& argmax, const at::Tensor& dx,
                 const c10::optional<at::Tensor>& gamma, const at::Tensor& save_mean, const at::Tensor& save_invstd,
                 const at::Tensor& ws, const c10::optional<at::Tensor>& dgamma,
                 const c10::optional<at::Tensor>& dbeta, bool grad_assign, const c10::optional<at::Tensor>& dy2,
                 int64_t pad, const c10::optional<at::Tensor>& xam) {
  check_dev(x, at::kBFloat16, "x");
  check_dev(dy, at::kBFloat16, "dy");
  check_dev(dx, at::kBFloat16, "dx");
  check_dev(argmax, at::kByte, "argmax");
  TORCH_CHECK(x.dim() == 4 && dy.dim() == 4 && x.is_contiguous() && dy.is_contiguous() && dx.is_contiguous() &&
                  dx.sizes() == x.sizes() && argmax.sizes() == dy.sizes() && argmax.is_contiguous() &&
                  dy.size(0) == x.size(0) && dy.size(3) == x.size(3),
              "bn_pool_bwd: dense NHWC tensors");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  ldnn::BnArgs a{};
  a.x = bf16_ptr(x);
  a.gamma = fptr_opt(gamma, C, "gamma");
  a.save_mean = fptr_opt(save_mean, C, "save_mean");
  a.save_invstd = fptr_opt(save_invstd, C, "save_invstd");
  a.ws = fptr_opt(ws, ldnn::bn_workspace_floats((int)C), "ws");
  a.M = (int)(N * H * W);
  a.C = (int)C;
  a.relu = 1;
  if (dy2.has_value()) {
    check_dev(*dy2, at::kBFloat16, "dy2");
    TORCH_CHECK(dy2->sizes() == dy.sizes() && dy2->is_contiguous(), "bn_pool_bwd: dy2 layout");
    a.dy2 = bf16_ptr(*dy2);
  }
  const uint8_t* am = argmax.data_ptr<uint8_t>();
  TORCH_CHECK(((uintptr_t)am & 7) == 0, "bn_pool_bwd: argmax must be 8-B aligned");
  const uint16_t* xam_p = nullptr;
  if (xam.has_value()) {
    check_dev(*xam, at::kBFloat16, "xam");
    TORCH_CHECK(xam->sizes() == dy.sizes() && xam->is_contiguous(), "bn_pool_bwd: xam must be laid out as dy");
    xam_p = bf16_ptr(*xam);
  }
  check(ldnn::bn_maxpool_backward(a, (int)N, (int)H, (int)W, (int)dy.size(1), (int)dy.size(2), (int)pad,
                                  bf16_ptr(dy), am, bf16_mut(dx), fptr_opt(dgamma, C, "dgamma"),
                                  fptr_opt(dbeta, C, "dbeta"), cur_stream(x), grad_assign, xam_p),
        "bn_maxpool_backward");
}

void gap_fwd(const at::Tensor& x, const at::Tensor& y) {  // x [N][HW][C], y [N][C]
  check_dev(x, at::kBFloat16, "x");
  check_dev(y, at::kBFloat16, "y");
  TORCH_CHECK(x.dim() == 3 && x.is_contiguous() && y.is_contiguous(), "gap: dense [N][HW][C]");
  check(ldnn::global_avgpool_fwd(bf16_ptr(x), bf16_mut(y), (int)x.size(0), (int)x.size(1), (int)x.size(2),
                                 cur_stream(x)),
        "gap_fwd");
}

void gap_bwd(const at::Tensor& dy, const at::Tensor& dx) {
  check_dev(dy, at::kBFloat16, "dy");
  check_dev(dx, at::kBFloat16, "dx");
  TORCH_CHECK(dx.dim() == 3 && dx.is_contiguous() && dy.is_contiguous(), "gap_bwd: dense");
  check(ldnn::global_avgpool_bwd(bf16_ptr(dy), bf16_mut(dx), (int)dx.size(0), (int)dx.size(1), (int)dx.size(2),
                                 cur_stream(dy)),
        "gap_bwd");
}


// x [N][HW][C] bf16, w [>= ncls][ldw] bf16, b [>= ncls] fp32 (optional) -> pooled [N][C], logits [N][>= ncls]
void gap_linear_fwd(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& b,
                    const at::Tensor& pooled, const at::Tensor& logits, int64_t ncls) {
  check_dev(x, at::kBFloat16, "x");
  check_dev(w, at::kBFloat16, "w");
  check_dev(pooled, at::kBFloat16, "pooled");
  check_dev(logits, at::kBFloat16, "logits");
  TORCH_CHECK(x.dim() == 3 && x.is_contiguous(), "gap_linear_fwd: x must be a dense [N][HW][C]");
  const int64_t N = x.size(0), HW = x.size(1), C = x.size(2);
  TORCH_CHECK(pooled.is_contiguous() && pooled.numel() == N * C, "gap_linear_fwd: pooled must be a dense [N][C]");
  TORCH_CHECK(w.dim() == 2 && w.stride(1) == 1 && w.size(0) >= ncls && w.size(1) >= C, "gap_linear_fwd: bad w");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1 && logits.size(0) == N && logits.size(1) >= ncls,
              "gap_linear_fwd: bad logits");
  TORCH_CHECK(ldnn::gap_linear_ok((int)N, (int)HW, (int)C, (int)ncls), "gap_linear_fwd: unsupported shape");
  const float* bp = nullptr;
  if (b.has_value()) {
    check_dev(*b, at::kFloat, "b");
    TORCH_CHECK(b->is_contiguous() && b->numel() >= ncls, "gap_linear_fwd: bad b");
    bp = b->data_ptr<float>();
  }
  check(ldnn::gap_linear_fwd(bf16_ptr(x), bf16_ptr(w), bp, bf16_mut(pooled), bf16_mut(logits), (int)N, (int)HW,
                             (int)C, (int)w.stride(0), (int)ncls, (int)logits.stride(0), cur_stream(x)),
        "gap_linear_fwd");
}

// g [N][>= ncls] bf16, pooled [N][C], w [>= ncls][ldw] -> dw [>= ncls][lddw] fp32 (beta_w), db (beta_b), dx [N][HW][C]
void gap_linear_bwd(const at::Tensor& g, const at::Tensor& pooled, const at::Tensor& w, const at::Tensor& dw,
                    const c10::optional<at::Tensor>& db, const at::Tensor& dx, int64_t ncls, double beta_w,
                    double beta_b) {
  check_dev(g, at::kBFloat16, "g");
  check_dev(pooled, at::kBFloat16, "pooled");
  check_dev(w, at::kBFloat16, "w");
  check_dev(dw, at::kFloat, "dw");
  check_dev(dx, at::kBFloat16, "dx");
  TORCH_CHECK(dx.dim() == 3 && dx.is_contiguous(), "gap_linear_bwd: dx must be a dense [N][HW][C]");
  const int64_t N = dx.size(0), HW = dx.size(1), C = dx.size(2);
  TORCH_CHECK(pooled.is_contiguous() && pooled.numel() == N * C, "gap_linear_bwd: pooled must be a dense [N][C]");
  TORCH_CHECK(g.dim() == 2 && g.stride(1) == 1 && g.size(0) == N && g.size(1) >= ncls, "gap_linear_bwd: bad g");
  TORCH_CHECK(w.dim() == 2 && w.stride(1) == 1 && w.size(0) >= ncls && w.size(1) >= C, "gap_linear_bwd: bad w");
  TORCH_CHECK(dw.dim() == 2 && dw.stride(1) == 1 && dw.size(0) >= ncls && dw.size(1) >= C, "gap_linear_bwd: bad dw");
  TORCH_CHECK(ldnn::gap_linear_ok((int)N, (int)HW, (int)C, (int)ncls), "gap_linear_bwd: unsupported shape");
  float* dbp = nullptr;
  if (db.has_value()) {
    check_dev(*db, at::kFloat, "db");
    TORCH_CHECK(db->is_contiguous() && db->numel() >= ncls, "gap_linear_bwd: bad db");
    dbp = db->data_ptr<float>();
  }
  check(ldnn::gap_linear_bwd(bf16_ptr(g), bf16_ptr(pooled), bf16_ptr(w), dw.data_ptr<float>(), dbp, bf16_mut(dx),
                             (int)N, (int)HW, (int)C, (int)g.stride(0), (int)w.stride(0), (int)dw.stride(0), (int)ncls,
                             (float)beta_w, (float)beta_b, cur_stream(g)),
        "gap_linear_bwd");
}
}  // namespace

// A HIP event whose record inside a stream capture becomes an EXTERNAL event-record
// node of the graph (hipEventRecordExternal): a stream outside the graph can then
// wait on a point in the middle of a graph replay -- how GraphedDPStep starts a
// bucket's RCCL all-reduce while the rest of the backward graph still runs.
// (torch.cuda.Event(external=True) refuses ROCm; HIP itself supports the node.)
struct GraphEvent {
  hipEvent_t ev = nullptr;
  GraphEvent() { check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreateWithFlags"); }
  ~GraphEvent() {
    if (ev != nullptr) (void)hipEventDestroy(ev);
  }
  GraphEvent(const GraphEvent&) = delete;
  GraphEvent& operator=(const GraphEvent&) = delete;
  void record_external(uint64_t stream) {
    check(hipEventRecordWithFlags(ev, reinterpret_cast<hipStream_t>(stream), hipEventRecordExternal),
          "hipEventRecordWithFlags(external)");
  }
  void record(uint64_t stream) { check(hipEventRecord(ev, reinterpret_cast<hipStream_t>(stream)), "hipEventRecord"); }
  void wait(uint64_t stream) {
    check(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), ev, 0), "hipStreamWaitEvent");
  }
  bool query() {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipErrorNotReady) return false;
    check(e, "hipEventQuery");
    return true;
  }
};


// One-shot all-reduce communicator (ipc.hip): this rank's staging + signal regions,
// exported as IPC handles, and the peers' regions opened from theirs.
struct OneShotComm {
  int rank, world, dev;
  size_t half_bytes;
  char* data = nullptr;      // own staging region, 2 halves
  uint32_t* sig = nullptr;   // own signal region (uncached)
  int* err = nullptr;        // own error word (uncached)
  uint32_t* ctr = nullptr;   // own per-block epoch counters (device memory: graph-replay safe)
  ldnn::IpcPeers peers{};
  std::vector<void*> opened;
  uint64_t calls = 0;        // host-side count of launches (diagnostics only)
  int blocks;

  OneShotComm(int rank_, int world_, int64_t max_bytes, int device, int blocks_)
      : rank(rank_), world(world_), dev(device), blocks(blocks_) {
    TORCH_CHECK(world >= 1 && world <= ldnn::kIpcMaxRanks && rank >= 0 && rank < world, "bad rank / world");
    TORCH_CHECK(blocks >= 1 && blocks <= ldnn::kIpcMaxBlocks, "blocks must be in [1, ", ldnn::kIpcMaxBlocks, "]");
    half_bytes = (size_t)((max_bytes + 255) / 256 * 256);
    check(hipSetDevice(dev), "hipSetDevice");
    check(hipMalloc(reinterpret_cast<void**>(&data), 2 * half_bytes), "hipMalloc(staging)");
    const size_t sbytes = sizeof(uint32_t) * ldnn::kIpcMaxBlocks * ldnn::kIpcMaxRanks;
    check(hipExtMallocWithFlags(reinterpret_cast<void**>(&sig), sbytes, hipDeviceMallocUncached), "hipExtMalloc(signals)");
    check(hipMemset(sig, 0, sbytes), "hipMemset(signals)");
    check(hipExtMallocWithFlags(reinterpret_cast<void**>(&err), 256, hipDeviceMallocUncached), "hipExtMalloc(err)");
    check(hipMemset(err, 0, 256), "hipMemset(err)");
    check(hipMalloc(reinterpret_cast<void**>(&ctr), sizeof(uint32_t) * ldnn::kIpcMaxBlocks), "hipMalloc(ctr)");
    check(hipMemset(ctr, 0, sizeof(uint32_t) * ldnn::kIpcMaxBlocks), "hipMemset(ctr)");
    check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    peers.half_bytes = half_bytes;
    peers.err = err;
    peers.mine = data;
    peers.ctr = ctr;
  }
  ~OneShotComm() {
    for (void* q : opened) (void)hipIpcCloseMemHandle(q);
    if (data) (void)hipFree(data);
    if (sig) (void)hipFree(sig);
    if (err) (void)hipFree(err);
    if (ctr) (void)hipFree(ctr);
  }
  static py::bytes handle_of(void* p) {
    hipIpcMemHandle_t h;
    check(hipIpcGetMemHandle(&h, p), "hipIpcGetMemHandle");
    return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  }
  py::tuple handles() const { return py::make_tuple(handle_of(data), handle_of(sig)); }
  // handles[j] = (staging handle, signal handle) of rank j (this rank's own entry is ignored)
  void connect(const std::vector<std::pair<std::string, std::string>>& hs) {
    TORCH_CHECK((int)hs.size() == world, "need one handle pair per rank");
    check(hipSetDevice(dev), "hipSetDevice");
    for (int j = 0; j < world; ++j) {
      if (j == rank) {
        peers.data[j] = data;
        peers.sig[j] = sig;
        continue;
      }
      void* ptrs[2];
      for (int k = 0; k < 2; ++k) {
        const std::string& b = k == 0 ? hs[j].first : hs[j].second;
        TORCH_CHECK(b.size() == sizeof(hipIpcMemHandle_t), "bad IPC handle size");
        hipIpcMemHandle_t h;
        std::memcpy(&h, b.data(), sizeof(h));
        check(hipIpcOpenMemHandle(&ptrs[k], h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
        opened.push_back(ptrs[k]);
      }
      peers.data[j] = reinterpret_cast<const char*>(ptrs[0]);
      peers.sig[j] = reinterpret_cast<uint32_t*>(ptrs[1]);
    }
  }
  // t <- sum over ranks of t (in place); fp32 or bf16, numel % 8 == 0, <= max_bytes
  void all_reduce(at::Tensor t) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "all_reduce needs a contiguous GPU tensor");
    const bool bf16 = t.scalar_type() == at::kBFloat16;
    TORCH_CHECK(bf16 || t.scalar_type() == at::kFloat, "fp32 or bf16 only");
    TORCH_CHECK(t.numel() % 8 == 0, "numel must be a multiple of 8");
    const size_t bytes = (size_t)t.numel() * t.element_size();
    TORCH_CHECK(bytes <= half_bytes, "tensor larger than the staging buffer");
    hipStream_t s = cur_stream(t);
    ++calls;
    check(ldnn::oneshot_all_reduce(peers, rank, world, t.numel(), bf16, t.data_ptr(), blocks, s),
          "oneshot_all_reduce");
  }
  // sticky error word (1: some call timed out waiting for a peer; every later call
  // leaves its tensor unsummed).  Synchronises the device.
  int error() const {
    int v = 0;
    check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    check(hipMemcpy(&v, err, sizeof(int), hipMemcpyDeviceToHost), "hipMemcpy(err)");
    return v;
  }
};

PYBIND11_MODULE(_C, m) {
  py::class_<GraphEvent>(m, "GraphEvent")
      .def(py::init<>())
      .def("record_external", &GraphEvent::record_external, py::arg("stream"),
           "record on a raw hipStream_t; inside a capture this is an external event-record node")
      .def("record", &GraphEvent::record, py::arg("stream"))
      .def("wait", &GraphEvent::wait, py::arg("stream"), "make the raw hipStream_t wait for the last record")
      .def("query", &GraphEvent::query);
  py::class_<OneShotComm>(m, "OneShotComm")
      .def(py::init<int, int, int64_t, int, int>(), py::arg("rank"), py::arg("world"), py::arg("max_bytes"),
           py::arg("device"), py::arg("blocks") = 64)
      .def("handles", &OneShotComm::handles, "(staging, signal) IPC handles of this rank")
      .def("connect", &OneShotComm::connect, py::arg("handles"))
      .def("all_reduce", &OneShotComm::all_reduce, py::arg("t"), "in-place sum over ranks (one kernel, one barrier)")
      .def("error", &OneShotComm::error)
      .def_readonly("calls", &OneShotComm::calls)
      .def_readonly("half_bytes", &OneShotComm::half_bytes);
  m.doc() = "ldnn: hand-written gfx950 (MI355X / CDNA4) HIP kernels";
  m.attr("EPI_NONE") = (int)ldnn::EPI_NONE;
  m.attr("EPI_BIAS") = (int)ldnn::EPI_BIAS;
  m.attr("EPI_BIAS_RELU") = (int)ldnn::EPI_BIAS_RELU;
  m.attr("EPI_BIAS_SIGMOID") = (int)ldnn::EPI_BIAS_SIGMOID;
  m.attr("EPI_DRELU") = (int)ldnn::EPI_DRELU;
  m.attr("EPI_DSIGMOID") = (int)ldnn::EPI_DSIGMOID;
  m.attr("ACT_RELU") = (int)ldnn::ACT_RELU;
  m.attr("ACT_SIGMOID") = (int)ldnn::ACT_SIGMOID;
  m.def("gemm", &gemm, "bf16 MFMA GEMM with fused epilogue", py::arg("a"), py::arg("b"), py::arg("c"),
        py::arg("a_kcontig"), py::arg("b_kcontig"), py::arg("epi") = 0, py::arg("bias") = py::none(),
        py::arg("aux") = py::none(), py::arg("dbias") = py::none(), py::arg("beta") = 0.0,
        py::arg("tile") = 0, py::arg("splitk") = 0, py::arg("direct_epi") = false, py::arg("variant") = 0,
        py::arg("ws") = py::none(), py::arg("cnt") = py::none(), py::arg("mask_out") = py::none(),
        py::arg("mask_in") = py::none(), py::arg("head_w") = py::none(), py::arg("head_part") = py::none());
  m.def("nchw_to_nhwc", [](const at::Tensor& src, const at::Tensor& dst, const c10::optional<at::Tensor>& extra_src,
                           const c10::optional<at::Tensor>& extra_dst, const c10::optional<at::Tensor>& s2d) {
        TORCH_CHECK(src.is_cuda() && src.dim() == 4 && src.is_contiguous() &&
                        (src.scalar_type() == at::kFloat || src.scalar_type() == at::kBFloat16),
                    "nchw_to_nhwc: src must be a contiguous NCHW fp32 / bf16 CUDA tensor");
        check_dev(dst, at::kBFloat16, "dst");
        const int64_t N = src.size(0), C = src.size(1), H = src.size(2), W = src.size(3);
        TORCH_CHECK(dst.dim() == 4 && dst.is_contiguous() && dst.size(0) == N && dst.size(1) == H && dst.size(2) == W &&
                        dst.size(3) >= C && dst.size(3) % 8 == 0 && aligned16(dst.data_ptr()),
                    "nchw_to_nhwc: dst must be contiguous [N][H][W][cp], cp >= C, cp % 8 == 0");
        const void* es = nullptr;
        void* ed = nullptr;
        int64_t eb = 0;
        if (extra_src.has_value() || extra_dst.has_value()) {   // e.g. the batch's labels, copied in the same launch
          TORCH_CHECK(extra_src.has_value() && extra_dst.has_value() && extra_src->is_cuda() && extra_dst->is_cuda() &&
                          extra_src->is_contiguous() && extra_dst->is_contiguous() &&
                          extra_src->nbytes() == extra_dst->nbytes() && extra_src->nbytes() % 8 == 0 &&
                          ((uintptr_t)extra_src->data_ptr() & 7) == 0 && ((uintptr_t)extra_dst->data_ptr() & 7) == 0,
                      "nchw_to_nhwc: extra_src / extra_dst must be contiguous GPU tensors of the same size, 8-B multiples");
          es = extra_src->data_ptr();
          ed = extra_dst->data_ptr();
          eb = (int64_t)extra_src->nbytes();
        }
        c10::hip::HIPGuardMasqueradingAsCUDA g(src.device());
        if (s2d.has_value()) {   // also the stem's space-to-depth image (conv_fwd(s2d_xs=..., s2d_packed=True))
          check_dev(*s2d, at::kBFloat16, "s2d");
          TORCH_CHECK(C <= 4 && dst.size(3) == 8 && H % 2 == 0 && W % 2 == 0 && s2d->is_contiguous() && s2d->dim() == 4 &&
                          s2d->size(0) == N && s2d->size(1) == H / 2 + 3 && s2d->size(2) == W / 2 + 3 &&
                          s2d->size(3) == 16 && aligned16(s2d->data_ptr()) &&
                          ((uintptr_t)src.data_ptr() % (src.scalar_type() == at::kFloat ? 8 : 4)) == 0,
                      "nchw_to_nhwc: s2d needs C <= 4, an 8-channel dst, even H and W and a dense "
                      "[N][H/2+3][W/2+3][16] bf16 image");
          check(ldnn::nchw_to_nhwc_s2d(src.data_ptr(), src.scalar_type() == at::kFloat, bf16_mut(dst), bf16_mut(*s2d),
                                       (int)N, (int)C, (int)H, (int)W, cur_stream(src), es, ed, eb),
                "nchw_to_nhwc_s2d");
          return;
        }
        check(ldnn::nchw_to_nhwc(src.data_ptr(), src.scalar_type() == at::kFloat, bf16_mut(dst), (int)N, (int)C,
                                 (int)(H * W), (int)dst.size(3), cur_stream(src), es, ed, eb),
              "nchw_to_nhwc");
      }, "NCHW fp32/bf16 -> NHWC bf16 with zeroed pad channels (+ an extra same-launch copy, e.g. labels; + the "
         "7x7 / 2 stem's packed space-to-depth image when s2d is given)",
      py::arg("src"), py::arg("dst"), py::arg("extra_src") = py::none(), py::arg("extra_dst") = py::none(),
      py::arg("s2d") = py::none());
  m.def("transpose_bf16", [](const at::Tensor& in, const at::Tensor& out) {
        check_dev(in, at::kBFloat16, "in");
        check_dev(out, at::kBFloat16, "out");
        TORCH_CHECK(in.dim() == 2 && out.dim() == 2 && out.size(0) == in.size(1) && out.size(1) == in.size(0),
                    "transpose_bf16: out must be [cols][rows] of in");
        const int64_t ldi = ld_of(in, "in"), ldo = ld_of(out, "out");
        TORCH_CHECK(in.size(0) % 8 == 0 && in.size(1) % 8 == 0 && ldi % 8 == 0 && ldo % 8 == 0 &&
                        aligned16(in.data_ptr()) && aligned16(out.data_ptr()),
                    "transpose_bf16: dims / strides must be multiples of 8, pointers 16-B aligned");
        c10::hip::HIPGuardMasqueradingAsCUDA g(in.device());
        check(ldnn::transpose_bf16(bf16_ptr(in), bf16_mut(out), (int)in.size(0), (int)in.size(1), (int)ldi, (int)ldo,
                                   cur_stream(in)), "transpose_bf16");
      }, "out = in^T (bf16)", py::arg("in"), py::arg("out"));
  m.def("slab_sum_cols", [](const at::Tensor& ws, const at::Tensor& out, const c10::optional<at::Tensor>& extra) {
        // ws [splits][rows][ldw] fp32 -> out [rows][ncols] (+ extra[rows] = column ncols of the sum)
        check_dev(ws, at::kFloat, "ws");
        check_dev(out, at::kFloat, "out");
        TORCH_CHECK(ws.dim() == 3 && ws.is_contiguous() && out.dim() == 2 && out.size(0) == ws.size(1) &&
                        out.stride(1) == 1 && aligned16(ws.data_ptr()), "slab_sum_cols: bad shapes");
        float* ex = nullptr;
        if (extra.has_value()) {
          check_dev(*extra, at::kFloat, "extra");
          TORCH_CHECK(extra->is_contiguous() && extra->numel() >= ws.size(1), "slab_sum_cols: bad extra");
          ex = extra->data_ptr<float>();
        }
        c10::hip::HIPGuardMasqueradingAsCUDA g(ws.device());
        check(ldnn::slab_sum_cols(ws.data_ptr<float>(), (int)ws.size(0), (int)ws.size(1), (int)ws.size(2),
                                  out.data_ptr<float>(), (int)out.stride(0), (int)out.size(1), ex, cur_stream(ws)),
              "slab_sum_cols");
      }, "sum split-K slabs into out (and one extra column)", py::arg("ws"), py::arg("out"),
      py::arg("extra") = py::none());
  m.def("slab_sum", [](const at::Tensor& ws, const at::Tensor& out, double beta) {
        // out = sum over the leading dim of ws (+ beta * out); fp32, dense, same trailing size
        check_dev(ws, at::kFloat, "ws");
        check_dev(out, at::kFloat, "out");
        TORCH_CHECK(ws.is_contiguous() && out.is_contiguous() && ws.dim() >= 2 && ws[0].numel() == out.numel() &&
                        out.numel() % 4 == 0 && aligned16(ws.data_ptr()) && aligned16(out.data_ptr()),
                    "slab_sum: ws must be a dense [splits][...] fp32 tensor matching the dense out");
        c10::hip::HIPGuardMasqueradingAsCUDA g(ws.device());
        check(ldnn::slab_sum(ws.data_ptr<float>(), out.data_ptr<float>(), out.numel() / 4, (int)ws.size(0),
                             (float)beta, cur_stream(ws)), "slab_sum");
      }, "sum of split-K partial slabs", py::arg("ws"), py::arg("out"), py::arg("beta") = 0.0);
  m.def("gemm_splitk_ws", [](int64_t M, int64_t N, int64_t splitk) {
        return std::make_pair((int64_t)(ldnn::gemm_splitk_ws_bytes((int)M, (int)N, (int)splitk) / 4),
                              (int64_t)ldnn::gemm_tiles128((int)M, (int)N));
      }, "(fp32 workspace elements, int32 counters) of a 128-tile split-K combine", py::arg("M"), py::arg("N"),
      py::arg("splitk"));
  m.def("gemm_q_ws", [](int64_t M, int64_t N, int64_t splitk) {
        return std::make_pair((int64_t)(ldnn::gemm_q_ws_bytes((int)M, (int)N, (int)splitk) / 4),
                              (int64_t)ldnn::gemm_q_tiles((int)M, (int)N));
      }, "(fp32 workspace elements, int32 counters) of a ping-pong 256-tile split-K combine", py::arg("M"),
      py::arg("N"), py::arg("splitk"));
  m.def("set_conv_impl", &ldnn::set_conv_impl, "0 = LDS-DMA fast path where it applies, 1 = generic kernel only",
        py::arg("impl"));
  m.def("set_conv_stem_s2d", &ldnn::set_conv_stem_s2d, "A/B: 1 = space-to-depth stem wgrad (default), 0 = off",
        py::arg("mode"));
  m.def("set_conv_wgrad_ring", &ldnn::set_conv_wgrad_ring, "A/B: ring wgrad for 3x3 stride-1 convs: 1 = 64x64 layers (default), 2 = every eligible shape, 0 = off",
        py::arg("mode"));
  m.def("set_conv_halo", &ldnn::set_conv_halo,
        "halo-staged 3x3 stride-1 conv: 0 off, 1 default (dgrad + 256x64 fwd tiles), 2 every eligible shape",
        py::arg("mode"));
  m.def("get_conv_halo", &ldnn::get_conv_halo);
  m.def("set_conv_hb", &ldnn::set_conv_hb,
        "big-tile (256x128, 8-wave) halo 3x3 stride-1 conv for 128-multiple output channels: 0 off, 1 on (default)",
        py::arg("mode"));
  m.def("get_conv_hb", &ldnn::get_conv_hb);
  m.def("set_conv_ws", &ldnn::set_conv_ws,
        "weight-stationary 64 -> 64 channel 3x3 stride-1 conv (fwd without bias, dgrad): 0 off, 1 on (default)",
        py::arg("mode"));
  m.def("get_conv_ws", &ldnn::get_conv_ws);
  m.def("set_conv_trace", [](const c10::optional<at::Tensor>& buf) {
        if (!buf.has_value()) {
          ldnn::set_conv_trace(nullptr);
          return;
        }
        TORCH_CHECK(buf->is_cuda() && buf->scalar_type() == at::kLong && buf->is_contiguous(), "set_conv_trace: int64 cuda");
        ldnn::set_conv_trace(reinterpret_cast<uint64_t*>(buf->data_ptr<int64_t>()));
      }, "phase-trace buffer of the LDNN_CONV_XF=32 diagnostic conv build ([>= workgroups][4] int64; None = off)",
      py::arg("buf"));
  m.def("get_conv_impl", &ldnn::get_conv_impl);
  m.def("gemm_opt", &gemm_opt, "weight-gradient GEMM with the optimizer update fused into its epilogue",
        py::arg("a"), py::arg("b"), py::arg("master"), py::arg("a_kcontig"), py::arg("b_kcontig"), py::arg("kind"),
        py::arg("m") = py::none(), py::arg("v") = py::none(), py::arg("shadow") = py::none(), py::arg("hp"),
        py::arg("grad_scale") = 1.0, py::arg("momentum") = 0.0, py::arg("dampening") = 0.0,
        py::arg("weight_decay") = 0.0, py::arg("nesterov") = false, py::arg("beta1") = 0.9, py::arg("beta2") = 0.999,
        py::arg("eps") = 1e-8, py::arg("tile") = 0, py::arg("splitk") = 0, py::arg("ws") = py::none(),
        py::arg("cnt") = py::none());
  m.def("act_fwd", &act_fwd);
  m.def("act_bwd", &act_bwd);
  m.def("colsum", &colsum, py::arg("x"), py::arg("out"), py::arg("accumulate") = false, py::arg("ws") = py::none());
  m.def("act_bwd_colsum", &act_bwd_colsum, py::arg("dy"), py::arg("y"), py::arg("dx"), py::arg("out"),
        py::arg("act"), py::arg("accumulate") = true, py::arg("ws") = py::none());
  m.def("cast_f32_bf16", &cast_f32_bf16);
  m.def("cast_bf16_f32", &cast_bf16_f32);
  m.def("mix3", &mix3, py::arg("out"), py::arg("x"), py::arg("y1") = py::none(), py::arg("y2") = py::none(),
        py::arg("a") = 1.0, py::arg("b") = 0.0, py::arg("c") = 0.0, py::arg("shadow") = py::none());
  m.def("softmax_xent", &softmax_xent, py::arg("logits"), py::arg("labels"), py::arg("dlogits"),
        py::arg("stats"), py::arg("dbias") = py::none(), py::arg("num_classes"), py::arg("grad_scale"),
        py::arg("loss_out") = py::none(), py::arg("loss_scale") = 1.0,
        "fused softmax-xent + argmax; loss_out: the last block writes [loss_sum * loss_scale, #correct] there "
        "(and adds both into stats if given)");
  m.def("scale_bf16", [](const at::Tensor& src, const at::Tensor& scale, const at::Tensor& out) {
    check_dev(src, at::kBFloat16, "src");
    check_dev(out, at::kBFloat16, "out");
    check_dev(scale, at::kFloat, "scale");
    TORCH_CHECK(src.is_contiguous() && out.is_contiguous() && src.numel() == out.numel() && scale.numel() >= 1,
                "scale_bf16: dense tensors of one size");
    c10::hip::HIPGuardMasqueradingAsCUDA g(src.device());
    check(ldnn::scale_bf16_dev(bf16_ptr(src), scale.data_ptr<float>(), bf16_mut(out), src.numel(), cur_stream(src)),
          "scale_bf16");
  }, py::arg("src"), py::arg("scale"), py::arg("out"), "out = src * scale[0] (device scalar)");
  m.def("standin_copy", [](const at::Tensor& src, const at::Tensor& dst, int64_t blocks, int64_t reps) {
    check_dev(src, at::kFloat, "src");
    check_dev(dst, at::kFloat, "dst");
    TORCH_CHECK(src.is_contiguous() && dst.is_contiguous() && src.numel() == dst.numel() && src.numel() % 4 == 0 &&
                    aligned16(src.data_ptr()) && aligned16(dst.data_ptr()),
                "standin_copy: dense, 16-B aligned fp32 tensors of one size, numel % 4 == 0");
    c10::hip::HIPGuardMasqueradingAsCUDA g(src.device());
    check(ldnn::standin_copy(src.data_ptr<float>(), dst.data_ptr<float>(), src.numel(), (int)blocks, (int)reps,
                             cur_stream(src)),
          "standin_copy");
  }, py::arg("src"), py::arg("dst"), py::arg("blocks"), py::arg("reps"),
        "overlap probe: reps copies of src into dst on `blocks` workgroups (an RCCL-sized footprint)");
  // roctx ranges (rocprofv3 --marker-trace shows them on the timeline)
  m.def("trace_push", [](const std::string& s) { return roctxRangePushA(s.c_str()); }, py::arg("name"));
  m.def("trace_pop", []() { return roctxRangePop(); });
  m.def("trace_mark", [](const std::string& s) { roctxMarkA(s.c_str()); }, py::arg("name"));
  m.def("trace_name_thread", [](const std::string& s) { roctxNameOsThread(s.c_str()); }, py::arg("name"));
  m.def(
      "gemm_plan",
      [](int64_t M, int64_t N, int64_t K, bool out_f32) {
        const int tile = ldnn::gemm_pick_tile((int)M, (int)N, (int)K, out_f32);
        return std::make_pair(tile, tile == 128 ? ldnn::gemm_pick_splitk((int)M, (int)N, (int)K) : 1);
      },
      "(tile, splitk) the auto dispatch picks for a (M, N, K) GEMM", py::arg("M"), py::arg("N"), py::arg("K"),
      py::arg("out_f32"));
  m.def("sgd_step", &sgd_step, py::arg("param"), py::arg("grad"), py::arg("mom"), py::arg("shadow"),
        py::arg("hp"), py::arg("grad_scale"), py::arg("momentum"), py::arg("dampening"),
        py::arg("weight_decay"), py::arg("nesterov"), py::arg("first_step"),
        py::arg("zero_ranges") = std::vector<std::pair<int64_t, int64_t>>{}, py::arg("t_begin") = 0,
        py::arg("t_out") = py::none());
  m.def("adam_step", &adam_step, py::arg("param"), py::arg("grad"), py::arg("m"), py::arg("v"),
        py::arg("shadow"), py::arg("hp"), py::arg("grad_scale"), py::arg("beta1"), py::arg("beta2"),
        py::arg("eps"), py::arg("weight_decay"), py::arg("decoupled"),
        py::arg("zero_ranges") = std::vector<std::pair<int64_t, int64_t>>{});
  m.def("bump_step", &bump_step);
  m.def("set_opt_max_blocks", &ldnn::set_opt_max_blocks, py::arg("n"),
        "grid cap of optimizer launches from now on (0 = default)");
  m.def("head_fwd_xent", &head_fwd_xent, "fused narrow Linear + softmax-xent + argmax (per-16-row stats slots)",
        py::arg("h"), py::arg("W"), py::arg("bias"), py::arg("labels"), py::arg("logits"), py::arg("dlogits"),
        py::arg("stats"), py::arg("num_classes"), py::arg("grad_scale"), py::arg("dh") = py::none(), py::arg("dbias") = py::none(),
        py::arg("dgrad_epi") = (int64_t)ldnn::EPI_DRELU, py::arg("dbias_ws") = py::none(),
        py::arg("dgrad_mode") = (int64_t)-1);
  m.def("head_dgrad_ws_floats", &ldnn::head_dgrad_ws_floats, py::arg("B"), py::arg("K"));
  m.def("head_xent_parts", &head_xent_parts, "softmax-xent + argmax from EPI_BIAS_RELU_HEAD partial logits",
        py::arg("parts"), py::arg("bias"), py::arg("labels"), py::arg("logits"), py::arg("dlogits"), py::arg("stats"),
        py::arg("num_classes"), py::arg("grad_scale"));
  m.def("head_dgrad_stream", &head_dgrad_stream, "streaming head dgrad: dh = (dlogits W) * act'(h), dbias += colsums",
        py::arg("h"), py::arg("W"), py::arg("dlogits"), py::arg("dh"), py::arg("dbias") = py::none(),
        py::arg("dgrad_epi") = (int64_t)ldnn::EPI_DRELU);
  m.def("head_bwd", &head_bwd, "fused head dgrad + wgrad (dW / db / dbias accumulated: pre-cleared)", py::arg("h"),
        py::arg("W"), py::arg("dlogits"), py::arg("dh"), py::arg("dW"), py::arg("dbias") = py::none(),
        py::arg("dgrad_epi") = (int64_t)ldnn::EPI_DRELU, py::arg("db") = py::none());
  m.def("head_wgrad", &head_wgrad, "dW = dz^T h (+ db = colsum dz); splits > 1 accumulate atomically",
        py::arg("dz"), py::arg("h"), py::arg("dW"), py::arg("db") = py::none(), py::arg("splits") = 0);
  m.def("head_dgrad_max_k", &ldnn::head_dgrad_max_k);
  m.def("head_wgrad_splits", &ldnn::head_wgrad_splits, py::arg("B"), py::arg("K"));
  m.def("bn_fwd", &bn_fwd, py::arg("x"), py::arg("y"), py::arg("residual"), py::arg("gamma"), py::arg("beta"),
        py::arg("running_mean"), py::arg("running_var"), py::arg("save_mean"), py::arg("save_invstd"),
        py::arg("ws"), py::arg("eps"), py::arg("momentum"), py::arg("training"), py::arg("relu"),
        py::arg("num_batches") = py::none(), py::arg("stats_ready") = false, py::arg("mask") = py::none());
  m.def("bn_workspace_floats", &ldnn::bn_workspace_floats, "fp32 workspace of one BatchNorm (zero it once, keep it)",
        py::arg("C"));
  m.def("bn_bwd", &bn_bwd, py::arg("x"), py::arg("y"), py::arg("dy"), py::arg("dx"), py::arg("dres"),
        py::arg("gamma"), py::arg("save_mean"), py::arg("save_invstd"), py::arg("ws"), py::arg("dgamma"),
        py::arg("dbeta"), py::arg("relu"), py::arg("mask") = py::none(), py::arg("grad_assign") = false,
        py::arg("dy2") = py::none(), py::arg("stats_ready") = false);
  m.def("pool_fwd", &pool_fwd, py::arg("x"), py::arg("y"), py::arg("argmax"), py::arg("R"), py::arg("S"),
        py::arg("stride"), py::arg("pad"), py::arg("is_max"), py::arg("nchw_out") = false);
  m.def("pool_bwd", &pool_bwd, py::arg("dy"), py::arg("argmax"), py::arg("dx"), py::arg("R"), py::arg("S"),
        py::arg("stride"), py::arg("pad"), py::arg("is_max"), py::arg("dy2") = py::none(),
        py::arg("nchw_dy") = false);
  m.def("bn_dual_fwd", &bn_dual_fwd, "y = relu(bn_a(x) + bn_b(r)) in one pass (the shortcut BN output never stored)",
        py::arg("x"), py::arg("r"), py::arg("y"), py::arg("mask"), py::arg("gamma_a"), py::arg("beta_a"),
        py::arg("rm_a"), py::arg("rv_a"), py::arg("mean_a"), py::arg("invstd_a"), py::arg("ws_a"), py::arg("eps_a"),
        py::arg("mom_a"), py::arg("nb_a"), py::arg("ready_a"), py::arg("gamma_b"), py::arg("beta_b"),
        py::arg("rm_b"), py::arg("rv_b"), py::arg("mean_b"), py::arg("invstd_b"), py::arg("ws_b"), py::arg("eps_b"),
        py::arg("mom_b"), py::arg("nb_b"), py::arg("ready_b"));
  m.def("bn_dual_bwd", &bn_dual_bwd, "backward of bn_dual_fwd: dx, dr and both BNs' dgamma / dbeta",
        py::arg("x"), py::arg("r"), py::arg("y"), py::arg("mask"), py::arg("dy"), py::arg("dy2"), py::arg("dx"),
        py::arg("dr"), py::arg("gamma_a"), py::arg("mean_a"), py::arg("invstd_a"), py::arg("ws_a"),
        py::arg("dgamma_a"), py::arg("dbeta_a"), py::arg("assign_a"), py::arg("gamma_b"), py::arg("mean_b"),
        py::arg("invstd_b"), py::arg("ws_b"), py::arg("dgamma_b"), py::arg("dbeta_b"), py::arg("assign_b"));
  m.def("bn_pool_fwd", &bn_pool_fwd, "relu(BN(x)) -> 3x3/2 max-pool in one pass (pooled output + argmax)",
        py::arg("x"), py::arg("y"), py::arg("argmax"), py::arg("gamma"), py::arg("beta"), py::arg("running_mean"),
        py::arg("running_var"), py::arg("save_mean"), py::arg("save_invstd"), py::arg("ws"), py::arg("eps"),
        py::arg("momentum"), py::arg("num_batches") = py::none(), py::arg("stats_ready") = false,
        py::arg("pad") = 1, py::arg("xam") = py::none());
  m.def("bn_pool_bwd", &bn_pool_bwd, "backward of bn_pool_fwd: dx, dgamma / dbeta", py::arg("x"), py::arg("dy"),
        py::arg("argmax"), py::arg("dx"), py::arg("gamma"), py::arg("save_mean"), py::arg("save_invstd"),
        py::arg("ws"), py::arg("dgamma"), py::arg("dbeta"), py::arg("grad_assign") = false,
        py::arg("dy2") = py::none(), py::arg("pad") = 1, py::arg("xam") = py::none());
  m.def("gap_fwd", &gap_fwd);
  m.def("gap_bwd", &gap_bwd);
  m.def("set_conv_combine_last", &ldnn::set_conv_combine_last,
        "split-K combine summer: 1 = the tile's last K slice, 0 = the last workgroup to arrive", py::arg("on"));
  m.def("get_conv_combine_last", &ldnn::get_conv_combine_last);
  m.def("set_conv_bn_bwd", &ldnn::set_conv_bn_bwd,
        "dgrad-side BN backward statistics: 0 off, 1 slab sum only (default), 2 also the dgrad epilogue");
  m.def("get_conv_bn_bwd", &ldnn::get_conv_bn_bwd);
  m.def("gap_linear_ok", &ldnn::gap_linear_ok, "shapes the fused pooled classifier head takes", py::arg("N"),
        py::arg("HW"), py::arg("C"), py::arg("ncls"));
  m.def("gap_linear_fwd", &gap_linear_fwd, "global average pool + Linear (<= 16 classes) in one launch", py::arg("x"),
        py::arg("w"), py::arg("b"), py::arg("pooled"), py::arg("logits"), py::arg("ncls"));
  m.def("gap_linear_bwd", &gap_linear_bwd, "its backward: dW, db and the input gradient in one launch", py::arg("g"),
        py::arg("pooled"), py::arg("w"), py::arg("dw"), py::arg("db"), py::arg("dx"), py::arg("ncls"),
        py::arg("beta_w") = 0.0, py::arg("beta_b") = 0.0);
  m.def("conv_fwd", &conv_fwd, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("stride"), py::arg("pad"),
        py::arg("bias") = py::none(), py::arg("epi") = 0, py::arg("bn_ws") = py::none(),
        py::arg("bn_gamma") = py::none(), py::arg("bn_beta") = py::none(), py::arg("bn_running_mean") = py::none(),
        py::arg("bn_running_var") = py::none(), py::arg("bn_save_mean") = py::none(),
        py::arg("bn_save_invstd") = py::none(), py::arg("bn_eps") = 1e-5, py::arg("bn_momentum") = 0.1,
        py::arg("bn_num_batches") = py::none(), py::arg("real_channels") = 0, py::arg("s2d_xs") = py::none(),
        py::arg("s2d_packed") = false);
  m.def("stem_s2d_fwd_ok", [](int64_t N, int64_t H, int64_t W, int64_t C, int64_t K, int64_t R, int64_t S,
                              int64_t stride, int64_t pad, int64_t real_channels) {
        ldnn::ConvShape s{};
        s.N = (int)N; s.H = (int)H; s.W = (int)W; s.C = (int)C; s.K = (int)K; s.R = (int)R; s.S = (int)S;
        s.stride = (int)stride; s.pad = (int)pad;
        s.P = (int)((H + 2 * pad - R) / stride + 1); s.Q = (int)((W + 2 * pad - S) / stride + 1);
        s.c_real = real_channels > 0 && real_channels < C ? (int)real_channels : 0;
        return ldnn::get_conv_impl() == 0 && ldnn::stem_s2d_fwd_ok(s);
      }, "whether conv_fwd takes s2d_xs for this stem shape (the 7x7 / 2 stem on its space-to-depth image)",
      py::arg("N"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("K"), py::arg("R"), py::arg("S"),
      py::arg("stride"), py::arg("pad"), py::arg("real_channels"));
  m.def("conv_dgrad", &conv_dgrad, py::arg("dy"), py::arg("w"), py::arg("dx"), py::arg("stride"), py::arg("pad"),
        py::arg("bn_x") = py::none(), py::arg("bn_mask") = py::none(), py::arg("bn_ws") = py::none(),
        py::arg("bn_gamma") = py::none(), py::arg("bn_save_mean") = py::none(),
        py::arg("bn_save_invstd") = py::none(), py::arg("bn_dgamma") = py::none(), py::arg("bn_dbeta") = py::none(),
        py::arg("bn_assign") = false);
  m.def("conv_fwd2", &conv_fwd2, py::arg("x"), py::arg("w0"), py::arg("y0"), py::arg("stride0"), py::arg("pad0"),
        py::arg("w1"), py::arg("y1"), py::arg("stride1"), py::arg("pad1"), py::arg("bn0") = py::none(),
        py::arg("bn1") = py::none(),
        "two forward convs of one input in one launch where the kernels allow; returns the BN-statistics flags");
  m.def("conv_bwd2", &conv_bwd2, py::arg("x"), py::arg("dy0"), py::arg("w0"), py::arg("dx0"), py::arg("dw0"),
        py::arg("stride0"), py::arg("pad0"), py::arg("beta0"), py::arg("dy1"), py::arg("w1"), py::arg("dx1"),
        py::arg("dw1"), py::arg("stride1"), py::arg("pad1"), py::arg("beta1"), py::arg("real_channels") = 0,
        "two convs of one input x, backward (dgrads + wgrads) in one launch where the kernels allow");
  m.def("conv_bwd", &conv_bwd, py::arg("dy"), py::arg("w"), py::arg("dx"), py::arg("x"), py::arg("dw"),
        py::arg("stride"), py::arg("pad"), py::arg("beta") = 0.0, py::arg("real_channels") = 0,
        py::arg("bn_x") = py::none(), py::arg("bn_mask") = py::none(), py::arg("bn_ws") = py::none(),
        py::arg("bn_gamma") = py::none(), py::arg("bn_save_mean") = py::none(),
        py::arg("bn_save_invstd") = py::none(), py::arg("bn_dgamma") = py::none(), py::arg("bn_dbeta") = py::none(),
        py::arg("bn_assign") = false,
        "conv_dgrad + conv_wgrad of one layer (one launch where the kernels allow); returns conv_dgrad's flag");
  m.def("set_conv_pair", &ldnn::set_conv_pair, "dgrad + wgrad in one launch (1, default) or one by one (0)");
  m.def("get_conv_pair", &ldnn::get_conv_pair);
  m.def("conv_wgrad", &conv_wgrad, py::arg("dy"), py::arg("x"), py::arg("dw"), py::arg("stride"), py::arg("pad"),
        py::arg("beta") = 0.0, py::arg("real_channels") = 0, py::arg("s2d_xs") = py::none(),
        "real_channels: channels of x that carry data (the rest zero padding, e.g. 3 of a stem's 8); 0 = all; "
        "s2d_xs: the forward's packed space-to-depth image (conv_fwd(s2d_xs=...))");
  m.def("synth_normal", &synth_normal);
  m.def("synth_labels", &synth_labels);
  m.def("augment_batch", &augment_batch, "gather + AutoAugment / flip+crop + normalise (augment.hip)");
}
