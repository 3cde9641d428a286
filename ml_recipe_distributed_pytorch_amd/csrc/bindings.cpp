// PyTorch bindings of the gfx950 kernels + RCCL reducer.  The only translation unit that includes
// torch headers.  Every entry point validates device/dtype/contiguity/shape before launching — a
// hand-written kernel must never see an operand whose shape its grid does not assume.
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <limits>
#include <map>

#include "hq_kernels.h"
#include "hq_reducer.h"

namespace {

using at::Tensor;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check(const Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void check_opt(const c10::optional<Tensor>& t, at::ScalarType dt, const char* name) {
  if (t.has_value() && t->defined()) check(*t, dt, name);
}
template <typename T>
T* ptr(const Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }
template <typename T>
T* optr(const c10::optional<Tensor>& t) { return (t.has_value() && t->defined()) ? reinterpret_cast<T*>(t->data_ptr()) : nullptr; }

const auto BF16 = at::kBFloat16;
const auto F32 = at::kFloat;
const auto I64 = at::kLong;

HqOuts outs4(float* a, float* b = nullptr, float* c = nullptr, float* d = nullptr) { return HqOuts{{a, b, c, d}}; }

uint32_t u32(int64_t v) { return (uint32_t)(v & 0xFFFFFFFFll); }

// ------------------------------------------------------------------------------------ embedding
std::vector<Tensor> embed_fwd(Tensor ids, Tensor pids, Tensor tids, Tensor ww, Tensor wp, Tensor wt, Tensor gamma,
                              Tensor beta, double eps, double p, int64_t seed, int64_t opid) {
  check(ids, I64, "ids"); check(pids, I64, "pos_ids"); check(tids, I64, "type_ids");
  check(ww, BF16, "w_word"); check(wp, BF16, "w_pos"); check(wt, BF16, "w_type");
  check(gamma, F32, "gamma"); check(beta, F32, "beta");
  const int64_t T = ids.numel(), H = ww.size(1);
  TORCH_CHECK(pids.numel() == T && tids.numel() == T, "id length mismatch");
  TORCH_CHECK(wp.size(1) == H && wt.size(1) == H && gamma.numel() == H && beta.numel() == H, "hidden mismatch");
  TORCH_CHECK(H % 4 == 0 && H <= 2048, "hidden size must be a multiple of 4 and <= 2048");
  TORCH_CHECK(T * H < (int64_t)std::numeric_limits<uint32_t>::max(), "T*H exceeds 32-bit dropout index");
  c10::DeviceGuard g(ids.device());
  auto y = at::empty({T, H}, ww.options());
  auto mean = at::empty({T}, gamma.options());
  auto rstd = at::empty({T}, gamma.options());
  hq_embed_fwd(ptr<int64_t>(ids), ptr<int64_t>(pids), ptr<int64_t>(tids), ptr<uint16_t>(ww), ptr<uint16_t>(wp),
               ptr<uint16_t>(wt), ptr<float>(gamma), ptr<float>(beta), ptr<uint16_t>(y), ptr<float>(mean), ptr<float>(rstd),
               (int)T, (int)H, (float)eps, (float)p, u32(seed), u32(opid), (int)ww.size(0), (int)wp.size(0),
               (int)wt.size(0), cur_stream());
  return {y, mean, rstd};
}

void embed_bwd(Tensor dy, Tensor ids, Tensor pids, Tensor tids, Tensor ww, Tensor wp, Tensor wt, Tensor gamma, Tensor mean,
               Tensor rstd, double p, int64_t seed, int64_t opid, Tensor g_word, Tensor g_pos, Tensor g_type, Tensor g_gamma,
               Tensor g_beta, bool accumulate, int64_t pad_word, int64_t pad_pos, int64_t seq_len) {
  check(dy, BF16, "dy"); check(ids, I64, "ids"); check(pids, I64, "pos_ids"); check(tids, I64, "type_ids");
  check(ww, BF16, "w_word"); check(wp, BF16, "w_pos"); check(wt, BF16, "w_type"); check(gamma, F32, "gamma");
  check(mean, F32, "mean"); check(rstd, F32, "rstd");
  check(g_word, F32, "g_word"); check(g_pos, F32, "g_pos"); check(g_type, F32, "g_type");
  check(g_gamma, F32, "g_gamma"); check(g_beta, F32, "g_beta");
  const int64_t T = ids.numel(), H = ww.size(1);
  TORCH_CHECK(dy.size(0) == T && dy.size(1) == H, "dy shape");
  TORCH_CHECK(g_word.sizes() == ww.sizes() && g_pos.sizes() == wp.sizes() && g_type.sizes() == wt.sizes(), "grad shapes");
  const int n_types = (int)wt.size(0);
  c10::DeviceGuard g(dy.device());
  auto s = cur_stream();
  if (!accumulate) {
    hq_zero_f32(ptr<float>(g_word), (size_t)g_word.numel(), s);
    hq_zero_f32(ptr<float>(g_pos), (size_t)g_pos.numel(), s);
    if (n_types > 2) hq_zero_f32(ptr<float>(g_type), (size_t)g_type.numel(), s);
  }
  const int nb = hq_embed_bwd_partials((int)T, (int)seq_len);
  auto part = at::empty({nb, 4 * H}, gamma.options());
  const int V = (int)ww.size(0);
  const HqEmbScratchSizes zs = hq_embed_bwd_scratch((int)T, V, (int)seq_len, (int)wp.size(0));
  auto pairs = at::empty({4, T}, ids.options().dtype(at::kInt));
  auto sort_tmp = at::empty({(int64_t)std::max<size_t>(zs.sort_bytes, 1)}, ids.options().dtype(at::kByte));
  auto carry = at::empty({(int64_t)zs.chunks * 2, H}, gamma.options());
  auto ppart = at::empty({std::max<int64_t>(zs.pos_rows, 1), H}, gamma.options());
  int32_t* pr = pairs.data_ptr<int32_t>();
  const HqEmbScratch sc{pr, pr + T, pr + 2 * T, pr + 3 * T, sort_tmp.data_ptr(), zs.sort_bytes, ptr<float>(carry),
                        ptr<float>(ppart)};
  float* t0 = ptr<float>(g_type);
  HqOuts o = outs4(ptr<float>(g_gamma), ptr<float>(g_beta), n_types <= 2 ? t0 : nullptr,
                   n_types == 2 ? t0 + H : nullptr);
  hq_embed_bwd(ptr<uint16_t>(dy), ptr<int64_t>(ids), ptr<int64_t>(pids), ptr<int64_t>(tids), ptr<uint16_t>(ww),
               ptr<uint16_t>(wp), ptr<uint16_t>(wt), ptr<float>(gamma), ptr<float>(mean), ptr<float>(rstd),
               ptr<float>(g_word), ptr<float>(g_pos), t0, ptr<float>(part), o, (int)T, (int)H, n_types, (int)pad_word,
               (int)pad_pos, (float)p, u32(seed), u32(opid), accumulate, V, (int)wp.size(0), (int)seq_len, sc, s);
}

// ------------------------------------------------------------------ residual + dropout + LayerNorm
// With q8 (f32[4] delayed-scaling state of the consuming fp8 GEMM's input): also returns y as e4m3.
// resid = None: `a` already is z (EPI_BDR GEMM epilogue) -> returns {y, a, mean, rstd} without touching z
// store_z = false: z is not written (returned empty) — the backward then recomputes x̂ from y (ln_bwd beta=)
std::vector<Tensor> ln_fwd(Tensor a, c10::optional<Tensor> resid_opt, Tensor gamma, Tensor beta, double eps, double p,
                           int64_t seed, int64_t opid, c10::optional<Tensor> q8, int64_t phase, bool store_z) {
  const bool zin = !(resid_opt.has_value() && resid_opt->defined());
  check(a, BF16, "a"); check(gamma, F32, "gamma"); check(beta, F32, "beta");
  if (!zin) check(*resid_opt, BF16, "resid");
  TORCH_CHECK(a.dim() == 2 && (zin || a.sizes() == resid_opt->sizes()), "a/resid shape");
  const int64_t T = a.size(0), H = a.size(1);
  TORCH_CHECK(gamma.numel() == H && beta.numel() == H && H % 4 == 0 && H <= 2048, "hidden size");
  TORCH_CHECK(T * H < (int64_t)std::numeric_limits<uint32_t>::max(), "T*H exceeds 32-bit dropout index");
  const bool want8 = q8.has_value() && q8->defined();
  TORCH_CHECK(!(zin && want8), "ln_fwd: the z-in form has no e4m3 output");
  if (want8) {
    check(*q8, F32, "q8");
    TORCH_CHECK(q8->numel() == 4, "q8 must be the f32[4] delayed-scaling state");
  }
  c10::DeviceGuard g(a.device());
  auto y = at::empty_like(a);
  const bool wz = zin || store_z;
  auto z = zin ? a : (store_z ? at::empty_like(a) : at::empty({0}, a.options()));
  auto mean = at::empty({T}, gamma.options()), rstd = at::empty({T}, gamma.options());
  Tensor y8 = want8 ? at::empty({T, H}, a.options().dtype(at::kFloat8_e4m3fn)) : Tensor();
  hq_ln_fwd(ptr<uint16_t>(a), zin ? nullptr : ptr<uint16_t>(*resid_opt), ptr<float>(gamma), ptr<float>(beta),
            ptr<uint16_t>(y), (zin || !wz) ? nullptr : ptr<uint16_t>(z),
            ptr<float>(mean), ptr<float>(rstd), (int)T, (int)H, (float)eps, (float)p, u32(seed), u32(opid), cur_stream(),
            want8 ? reinterpret_cast<uint8_t*>(y8.data_ptr()) : nullptr, want8 ? ptr<float>(*q8) : nullptr,
            (int)(phase % 3));
  if (want8) return {y, z, mean, rstd, y8};
  return {y, z, mean, rstd};
}

// q8 (f32[4] delayed-scaling state of the fp8 dgrad GEMM that consumes da): also returns da as e5m2
std::vector<Tensor> ln_bwd(Tensor dy, c10::optional<Tensor> dy2, Tensor z, Tensor gamma, Tensor mean, Tensor rstd, double p,
                           int64_t seed, int64_t opid, c10::optional<Tensor> g_gamma, c10::optional<Tensor> g_beta,
                           c10::optional<Tensor> g_bias, bool accumulate, c10::optional<Tensor> q8, int64_t phase,
                           bool write_da, c10::optional<Tensor> beta) {
  // beta given: `z` is the forward OUTPUT y and x̂ = (y − β)/γ (the forward ran with store_z = false)
  const bool fromy = beta.has_value() && beta->defined();
  if (fromy) {
    check(*beta, F32, "beta");
    TORCH_CHECK(beta->numel() == dy.size(1), "ln_bwd: beta length");
  }
  check(dy, BF16, "dy"); check_opt(dy2, BF16, "dy2"); check(z, BF16, "z"); check(gamma, F32, "gamma");
  check(mean, F32, "mean"); check(rstd, F32, "rstd");
  check_opt(g_gamma, F32, "g_gamma"); check_opt(g_beta, F32, "g_beta"); check_opt(g_bias, F32, "g_bias");
  TORCH_CHECK(dy.sizes() == z.sizes(), "dy/z shape");
  if (dy2.has_value() && dy2->defined()) TORCH_CHECK(dy2->sizes() == dy.sizes(), "dy2 shape");
  const int64_t T = dy.size(0), H = dy.size(1);
  TORCH_CHECK(gamma.numel() == H && mean.numel() == T && rstd.numel() == T, "stat shapes");
  c10::DeviceGuard g(dy.device());
  // write_da = false (with q8): da only as e5m2 — the bf16 da comes back empty
  TORCH_CHECK(write_da || (q8.has_value() && q8->defined()), "ln_bwd: write_da=False needs q8");
  auto dz = at::empty_like(dy), da = write_da ? at::empty_like(dy) : at::empty({0}, dy.options());
  const int nb = hq_ln_bwd_partials((int)T);
  auto part = at::empty({nb, 3 * H}, gamma.options());
  const bool want8 = q8.has_value() && q8->defined();
  Tensor da8;
  if (want8) {
    check(*q8, F32, "q8");
    TORCH_CHECK(q8->numel() == 4, "ln_bwd: q8 must be f32[4]");
    TORCH_CHECK(H % 4 == 0, "ln_bwd: e5m2 output needs H % 4 == 0");
    da8 = at::empty(dy.sizes(), dy.options().dtype(at::kFloat8_e5m2));
  }
  hq_ln_bwd(ptr<uint16_t>(dy), optr<uint16_t>(dy2), ptr<uint16_t>(z), ptr<float>(gamma), ptr<float>(mean), ptr<float>(rstd),
            ptr<uint16_t>(dz), write_da ? ptr<uint16_t>(da) : nullptr, ptr<float>(part),
            outs4(optr<float>(g_gamma), optr<float>(g_beta), optr<float>(g_bias)), (int)T, (int)H, (float)p, u32(seed),
            u32(opid), accumulate, cur_stream(), want8 ? reinterpret_cast<uint8_t*>(da8.data_ptr()) : nullptr,
            want8 ? ptr<float>(*q8) : nullptr, (int)(phase % 3), fromy ? ptr<float>(*beta) : nullptr);
  if (want8) return {dz, da, da8};
  return {dz, da};
}

// ------------------------------------------------------------------------------------------ GELU
// ------------------------------------------------------------------------------------ MFMA GEMM
// C[M,N] = A[M,K] · B[N,K]^T with epilogue `epi` (HQ_EPI_*).  bias f32[N] (BIAS/GELU); pre bf16[M,N]
// (GELU: written, DGELU: read); resid bf16[M,N] (RESID); part f32[M/256, N] (DGELU column partials).
int64_t gemm_nt_supported(int64_t M, int64_t N, int64_t K) { return hq_gemm_nt_supported((int)M, (int)N, (int)K); }

Tensor gemm_nt(Tensor A, Tensor B, int64_t epi, c10::optional<Tensor> bias, c10::optional<Tensor> pre,
               c10::optional<Tensor> resid, c10::optional<Tensor> part, c10::optional<Tensor> out, double p, int64_t seed,
               int64_t opid) {
  check(A, BF16, "A"); check(B, BF16, "B");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(1) == B.size(1), "gemm_nt: A[M,K], B[N,K] expected");
  const int64_t M = A.size(0), K = A.size(1), N = B.size(0);
  TORCH_CHECK(M < (1ll << 31) / 4 && N * K < (1ll << 31) && M * N < (1ll << 40), "gemm_nt: shape too large");
  const int bn = hq_gemm_nt_supported((int)M, (int)N, (int)K);
  TORCH_CHECK(bn > 0, "gemm_nt: unsupported shape M=", M, " N=", N, " K=", K, " (need N%128, K%64 == 0)");
  TORCH_CHECK(epi >= HQ_EPI_NONE && epi <= HQ_EPI_BDR, "gemm_nt: bad epilogue");
  if (epi == HQ_EPI_BDR) {
    TORCH_CHECK(bias.has_value() && bias->defined(), "gemm_nt: EPI_BDR needs the fp32 bias");
    TORCH_CHECK(M * N < (int64_t)std::numeric_limits<uint32_t>::max(), "gemm_nt: M*N exceeds 32-bit dropout index");
  }
  c10::DeviceGuard g(A.device());
  Tensor C = (out.has_value() && out->defined()) ? *out : at::empty({M, N}, A.options());
  check(C, BF16, "out");
  TORCH_CHECK(C.size(0) == M && C.size(1) == N, "gemm_nt: out shape");
  if (epi == HQ_EPI_BIAS || epi == HQ_EPI_GELU || epi == HQ_EPI_GELUD) {
    TORCH_CHECK(bias.has_value() && bias->defined(), "gemm_nt: bias required");
    check(*bias, F32, "bias");
    TORCH_CHECK(bias->numel() == N, "gemm_nt: bias length");
  }
  if (epi == HQ_EPI_GELU || epi == HQ_EPI_DGELU || epi == HQ_EPI_GELUD || epi == HQ_EPI_DMUL) {
    TORCH_CHECK(pre.has_value() && pre->defined(), "gemm_nt: pre required");
    check(*pre, BF16, "pre");
    TORCH_CHECK(pre->size(0) == M && pre->size(1) == N, "gemm_nt: pre shape");
  }
  if (epi == HQ_EPI_RESID || epi == HQ_EPI_BDR) {
    TORCH_CHECK(resid.has_value() && resid->defined(), "gemm_nt: resid required");
    check(*resid, BF16, "resid");
    TORCH_CHECK(resid->size(0) == M && resid->size(1) == N, "gemm_nt: resid shape");
  }
  if (epi == HQ_EPI_DGELU || epi == HQ_EPI_DMUL) {
    TORCH_CHECK(part.has_value() && part->defined(), "gemm_nt: part required");
    check(*part, F32, "part");
    TORCH_CHECK(part->numel() == (int64_t)hq_gemm_nt_part_rows((int)M, (int)N, (int)K) * N,
                "gemm_nt: part must hold [gemm_nt_part_rows(M, N, K), N]");
  }
  // split-K slabs (128² kernel, low-fill long-K grids) from the stream-aware caching allocator: safe beside
  // other streams and inside graph captures once the shape has run eagerly
  const size_t wsf = hq_gemm_nt_ws_floats((int)M, (int)N, (int)K, (int)epi);
  Tensor ws = wsf ? at::empty({(int64_t)wsf}, A.options().dtype(at::kFloat)) : Tensor();
  hq_gemm_nt(ptr<uint16_t>(A), ptr<uint16_t>(B), ptr<uint16_t>(C), optr<float>(bias), optr<uint16_t>(pre),
             optr<uint16_t>(resid), optr<float>(part), (int)M, (int)N, (int)K, (int)K, (int)K, (int)N, (int)epi, bn,
             cur_stream(), (float)p, u32(seed), u32(opid), wsf ? ws.data_ptr<float>() : nullptr);
  return C;
}

// Weight gradient: out [N,K] f32 (+)= dyᵀ·x with dy [T,N], x [T,K] bf16; split-K slabs from the caching allocator.
int64_t gemm_tn_splits(int64_t T, int64_t N, int64_t K) { return hq_gemm_tn_splits((int)T, (int)N, (int)K); }

void gemm_tn(Tensor dy, Tensor x, Tensor out, bool accumulate, int64_t splits, c10::optional<Tensor> bias_out) {
  check(dy, BF16, "dy"); check(x, BF16, "x"); check(out, F32, "out");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && dy.size(0) == x.size(0), "gemm_tn: dy [T,N], x [T,K]");
  const int64_t T = dy.size(0), N = dy.size(1), K = x.size(1);
  TORCH_CHECK(out.numel() == N * K, "gemm_tn: out must hold N*K");
  const int auto_s = hq_gemm_tn_splits((int)T, (int)N, (int)K);
  TORCH_CHECK(auto_s > 0, "gemm_tn: unsupported shape T=", T, " N=", N, " K=", K, " (need N%128, K%128 == 0, T >= 128)");
  const int S = splits > 0 ? (int)splits : auto_s;
  TORCH_CHECK((T + 63) / 64 / S >= 2, "gemm_tn: too many splits");
  const bool has_bias = bias_out.has_value() && bias_out->defined();
  if (has_bias) {
    check(*bias_out, F32, "bias_out");
    TORCH_CHECK(bias_out->numel() == N, "gemm_tn: bias_out must hold N");
  }
  c10::DeviceGuard g(dy.device());
  Tensor part = at::empty({S, N, K}, out.options());
  Tensor bpart = has_bias ? at::empty({S, N}, out.options()) : Tensor();
  hq_gemm_tn(ptr<uint16_t>(dy), ptr<uint16_t>(x), ptr<float>(part), ptr<float>(out), has_bias ? ptr<float>(bpart) : nullptr,
             has_bias ? ptr<float>(*bias_out) : nullptr, (int)T, (int)N, (int)K, S, accumulate, cur_stream());
}

// --precision fp32: exact-f32 strided / batched GEMM (gemm_f32.hip).  C(z, i, j) = alpha·Σ_k A(z,i,k)·B(z,j,k)
// (+ bias[j]) (+ R(z,i,j)), every operand addressed from its tensor's data_ptr by the given strides — the bounds
// check below proves every element the grid touches lies inside its tensor's storage.
namespace {
void f32_span_check(const Tensor& t, const char* name, std::initializer_list<std::pair<int64_t, int64_t>> dims) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == F32, name, " must be a float32 GPU tensor");
  int64_t hi = 0;
  for (auto& d : dims) {
    TORCH_CHECK(d.first >= 1 && d.second >= 0, name, ": bad extent/stride");
    hi += (d.first - 1) * d.second;
  }
  const int64_t avail = (int64_t)(t.storage().nbytes() / 4) - t.storage_offset();
  TORCH_CHECK(hi < avail, name, ": strided extent ", hi + 1, " exceeds the tensor's storage (", avail, " floats)");
  TORCH_CHECK(((uintptr_t)t.data_ptr() & 15) == 0, name, " must be 16-byte aligned");
}
}  // namespace

void gemm_f32(Tensor A, Tensor B, Tensor C, int64_t M, int64_t N, int64_t K, std::vector<int64_t> sa,
              std::vector<int64_t> sb, std::vector<int64_t> sc, int64_t batch, int64_t nb_in, double alpha,
              c10::optional<Tensor> bias, c10::optional<Tensor> R, int64_t ldr) {
  // sa = {sa_i, sa_k, ba_out, ba_in}, sb = {sb_j, sb_k, bb_out, bb_in}, sc = {ldc, bc_out, bc_in}
  TORCH_CHECK(sa.size() == 4 && sb.size() == 4 && sc.size() == 3, "gemm_f32: stride vectors");
  TORCH_CHECK(M > 0 && N > 0 && K > 0 && batch >= 1 && nb_in >= 1 && batch % nb_in == 0, "gemm_f32: bad sizes");
  TORCH_CHECK(M * N < (int64_t)1 << 31 && K < (int64_t)1 << 31, "gemm_f32: sizes exceed 32-bit tile indexing");
  const int64_t nbo = batch / nb_in;
  TORCH_CHECK(sa[1] == 1 || sa[0] == 1, "gemm_f32: A needs a unit i or k stride");
  TORCH_CHECK(sb[1] == 1 || sb[0] == 1, "gemm_f32: B needs a unit j or k stride");
  // float4 staging: the contiguous extent is a multiple of 4 and the other stride keeps quads 16-B aligned
  if (sa[1] == 1) {
    TORCH_CHECK(K % 4 == 0 && sa[0] % 4 == 0, "gemm_f32: k-contiguous A needs K % 4 == 0, sa_i % 4 == 0");
  } else {
    TORCH_CHECK(M % 4 == 0 && sa[1] % 4 == 0, "gemm_f32: i-contiguous A needs M % 4 == 0, sa_k % 4 == 0");
  }
  if (sb[1] == 1) {
    TORCH_CHECK(K % 4 == 0 && sb[0] % 4 == 0, "gemm_f32: k-contiguous B needs K % 4 == 0, sb_j % 4 == 0");
  } else {
    TORCH_CHECK(N % 4 == 0 && sb[1] % 4 == 0, "gemm_f32: j-contiguous B needs N % 4 == 0, sb_k % 4 == 0");
  }
  TORCH_CHECK(sa[2] % 4 == 0 && sa[3] % 4 == 0 && sb[2] % 4 == 0 && sb[3] % 4 == 0, "gemm_f32: batch strides % 4");
  f32_span_check(A, "A", {{M, sa[0]}, {K, sa[1]}, {nbo, sa[2]}, {nb_in, sa[3]}});
  f32_span_check(B, "B", {{N, sb[0]}, {K, sb[1]}, {nbo, sb[2]}, {nb_in, sb[3]}});
  f32_span_check(C, "C", {{M, sc[0]}, {N, 1}, {nbo, sc[1]}, {nb_in, sc[2]}});
  const bool has_r = R.has_value() && R->defined();
  if (has_r) f32_span_check(*R, "R", {{M, ldr}, {N, 1}, {nbo, sc[1]}, {nb_in, sc[2]}});
  const bool has_b = bias.has_value() && bias->defined();
  if (has_b) { check(*bias, F32, "bias"); TORCH_CHECK(bias->numel() == N, "gemm_f32: bias must hold N"); }
  c10::DeviceGuard g(A.device());
  const int ks = hq_gemm_f32_splits((int)M, (int)N, (int)K, (int)batch);
  Tensor ws = ks > 1 ? at::empty({ks, M, N}, C.options()) : Tensor();
  hq_gemm_f32(ptr<float>(A), ptr<float>(B), ptr<float>(C), has_b ? ptr<float>(*bias) : nullptr,
              has_r ? ptr<float>(*R) : nullptr, ks > 1 ? ptr<float>(ws) : nullptr, (int)M, (int)N, (int)K, sa[0], sa[1],
              sb[0], sb[1], (int)sc[0], (int)ldr, (int)batch, (int)nb_in, sa[2], sa[3], sb[2], sb[3], sc[1], sc[2],
              (float)alpha, ks, cur_stream());
}

// fp8 weight gradient: out [N,K] f32 (+)= (dy8ᵀ·x8)·sa·sb, dy8 e5m2 [T,N], x8 e4m3 [T,K] (token-major)
int64_t gemm_tn8_splits(int64_t T, int64_t N, int64_t K) { return hq_gemm_tn8_splits((int)T, (int)N, (int)K); }

void gemm_tn8(Tensor dy8, Tensor x8, Tensor sa, Tensor sb, Tensor out, bool accumulate) {
  TORCH_CHECK(dy8.is_cuda() && dy8.scalar_type() == at::kFloat8_e5m2 && dy8.is_contiguous() && dy8.dim() == 2,
              "gemm_tn8: dy8 must be a contiguous float8_e5m2 [T,N] GPU tensor");
  TORCH_CHECK(x8.is_cuda() && x8.scalar_type() == at::kFloat8_e4m3fn && x8.is_contiguous() && x8.dim() == 2 &&
              x8.size(0) == dy8.size(0), "gemm_tn8: x8 must be a contiguous float8_e4m3fn [T,K] GPU tensor");
  check(out, F32, "out"); check(sa, F32, "sa"); check(sb, F32, "sb");
  const int64_t T = dy8.size(0), N = dy8.size(1), K = x8.size(1);
  TORCH_CHECK(out.numel() == N * K, "gemm_tn8: out must hold N*K");
  const int S = hq_gemm_tn8_splits((int)T, (int)N, (int)K);
  TORCH_CHECK(S > 0, "gemm_tn8: unsupported shape T=", T, " N=", N, " K=", K, " (need N%128, K%128 == 0)");
  c10::DeviceGuard g(dy8.device());
  Tensor part = at::empty({S, N, K}, out.options());
  hq_gemm_tn8(reinterpret_cast<const uint8_t*>(dy8.data_ptr()), reinterpret_cast<const uint8_t*>(x8.data_ptr()),
              ptr<float>(sa), ptr<float>(sb), ptr<float>(part), ptr<float>(out), (int)T, (int)N, (int)K, S, accumulate,
              cur_stream());
}

// fp8 projection GEMM, C (bf16) = A8·B8ᵀ·sa·sb (+ epilogue), B8 e4m3.  Forward (A8 e4m3): BIAS / GELUD
// (+ bias f32; GELUD returns act, writes gelu' into `pre` and, with out8/state given, act as e4m3).
// Backward dgrad (A8 e5m2): NONE / DMUL (C ⊙ pre, column sums into part [M/256, N]; with out8/state,
// C also as e5m2).  Delayed scaling: state f32[4], phase = step % 3.
int64_t gemm_fp8_supported(int64_t M, int64_t N, int64_t K) { return hq_gemm_fp8_supported((int)M, (int)N, (int)K); }

Tensor gemm_fp8(Tensor A8, Tensor B8, int64_t epi, c10::optional<Tensor> bias, Tensor sa, Tensor sb,
                c10::optional<Tensor> pre, c10::optional<Tensor> out8, c10::optional<Tensor> state, int64_t phase,
                c10::optional<Tensor> part, c10::optional<Tensor> resid, bool write_out) {
  TORCH_CHECK(A8.is_cuda() && A8.element_size() == 1 && A8.is_contiguous() && B8.is_cuda() && B8.element_size() == 1 &&
              B8.is_contiguous(), "gemm_fp8: A8 / B8 must be contiguous 1-byte (fp8) GPU tensors");
  TORCH_CHECK(A8.dim() == 2 && B8.dim() == 2 && A8.size(1) == B8.size(1), "gemm_fp8: A8[M,K], B8[N,K]");
  TORCH_CHECK(B8.scalar_type() == at::kFloat8_e4m3fn, "gemm_fp8: B8 (weights) must be float8_e4m3fn");
  const int64_t M = A8.size(0), K = A8.size(1), N = B8.size(0);
  TORCH_CHECK(hq_gemm_fp8_supported((int)M, (int)N, (int)K), "gemm_fp8: unsupported shape M=", M, " N=", N, " K=", K);
  const bool fwd = epi == HQ_EPI_BIAS || epi == HQ_EPI_GELUD;
  const bool bwd = epi == HQ_EPI_NONE || epi == HQ_EPI_DMUL || epi == HQ_EPI_RESID;
  TORCH_CHECK(fwd || bwd, "gemm_fp8: epilogue must be BIAS / GELUD (forward) or NONE / RESID / DMUL (dgrad)");
  TORCH_CHECK(A8.scalar_type() == (fwd ? at::kFloat8_e4m3fn : at::kFloat8_e5m2),
              "gemm_fp8: A8 must be float8_e4m3fn for the forward epilogues, float8_e5m2 for the dgrad ones");
  check(sa, F32, "sa"); check(sb, F32, "sb");
  TORCH_CHECK(sa.numel() >= 1 && sb.numel() >= 1, "gemm_fp8: sa, sb");
  if (fwd) {
    TORCH_CHECK(bias.has_value() && bias->defined(), "gemm_fp8: forward epilogues need the fp32 bias");
    check(*bias, F32, "bias");
    TORCH_CHECK(bias->numel() == N, "gemm_fp8: bias[N]");
  }
  c10::DeviceGuard g(A8.device());
  // write_out = false (GELUD / DMUL with out8): only the fp8 copy (and P / part) — returns an empty tensor
  TORCH_CHECK(write_out || ((epi == HQ_EPI_GELUD || epi == HQ_EPI_DMUL) && out8.has_value() && out8->defined()),
              "gemm_fp8: write_out=False needs a GELUD / DMUL epilogue with out8");
  Tensor C = write_out ? at::empty({M, N}, A8.options().dtype(BF16)) : at::empty({0}, A8.options().dtype(BF16));
  uint16_t* P = nullptr;
  uint8_t* C8 = nullptr;
  float* q8 = nullptr;
  float* pp = nullptr;
  bool code8 = true;
  if (epi == HQ_EPI_DMUL) {
    TORCH_CHECK(part.has_value() && part->defined(), "gemm_fp8: DMUL needs `part` [M/256, N]");
    check(*part, F32, "part");
    TORCH_CHECK(part->numel() == (M / 256) * N, "gemm_fp8: part must hold [M/256, N]");
    pp = ptr<float>(*part);
  }
  if (epi == HQ_EPI_RESID) {
    TORCH_CHECK(resid.has_value() && resid->defined(), "gemm_fp8: RESID needs `resid`");
    check(*resid, BF16, "resid");
    TORCH_CHECK(resid->size(0) == M && resid->size(1) == N, "gemm_fp8: resid shape");
    P = ptr<uint16_t>(*resid);
  }
  if (epi == HQ_EPI_GELUD || epi == HQ_EPI_DMUL) {
    TORCH_CHECK(pre.has_value() && pre->defined(), "gemm_fp8: GELUD / DMUL need `pre` (gelu')");
    // gelu' travels as the 8-bit code (hq_gd_encode8, a uint8 `pre`) between the fp8 FFN1 forward and the fp8
    // FFN2 dgrad, else as bf16.  The fp8 DMUL reads only the code; the fp8 GELUD writes bf16 gelu' (beside its
    // e4m3 act) only together with the bf16 act, i.e. when the backward will run the FFN2 dgrad in bf16.
    const bool with8 = out8.has_value() && out8->defined();
    code8 = pre->scalar_type() == at::kByte;
    if (code8) {
      TORCH_CHECK(with8 && pre->is_cuda() && pre->is_contiguous(),
                  "gemm_fp8: the uint8 gelu' code (gelud_code()) goes with out8");
    } else {
      check(*pre, BF16, "pre");
      TORCH_CHECK(!with8 || (epi == HQ_EPI_GELUD && write_out),
                  "gemm_fp8: a bf16 gelu' with out8 needs GELUD with write_out (fp8 DMUL reads the uint8 code)");
    }
    TORCH_CHECK(pre->size(0) == M && pre->size(1) == N, "gemm_fp8: pre shape");
    P = reinterpret_cast<uint16_t*>(pre->data_ptr());
    if (out8.has_value() && out8->defined()) {
      TORCH_CHECK(out8->scalar_type() == (fwd ? at::kFloat8_e4m3fn : at::kFloat8_e5m2),
                  "gemm_fp8: out8 must be float8_e4m3fn (GELUD) / float8_e5m2 (DMUL)");
      TORCH_CHECK(out8->is_cuda() && out8->element_size() == 1 && out8->is_contiguous() && out8->numel() == M * N,
                  "gemm_fp8: out8 must be a contiguous 1-byte [M,N] tensor");
      TORCH_CHECK(state.has_value() && state->defined(), "gemm_fp8: out8 needs the delayed-scaling state");
      check(*state, F32, "state");
      TORCH_CHECK(state->numel() == 4, "gemm_fp8: state must be f32[4]");
      C8 = reinterpret_cast<uint8_t*>(out8->data_ptr());
      q8 = ptr<float>(*state);
    }
  }
  hq_gemm_fp8(reinterpret_cast<const uint8_t*>(A8.data_ptr()), reinterpret_cast<const uint8_t*>(B8.data_ptr()),
              write_out ? ptr<uint16_t>(C) : nullptr,
              optr<float>(bias), P, ptr<float>(sa), ptr<float>(sb), C8, q8, (int)(phase % 3), (int)M, (int)N, (int)K,
              (int)epi, cur_stream(), pp, code8 ? 1 : 0);
  return C;
}

// x (bf16) -> e4m3 with the delayed scale of `state` (f32[4]); returns y (float8_e4m3fn); state[3] = scale
Tensor fp8_quant_delayed(Tensor x, Tensor state, int64_t phase) {
  check(x, BF16, "x"); check(state, F32, "state");
  TORCH_CHECK(x.numel() % 8 == 0 && state.numel() == 4, "fp8_quant_delayed: numel % 8 / state f32[4]");
  c10::DeviceGuard g(x.device());
  auto y = at::empty(x.sizes(), x.options().dtype(at::kFloat8_e4m3fn));
  hq_fp8_quant_delayed(ptr<uint16_t>(x), reinterpret_cast<uint8_t*>(y.data_ptr()), x.numel(), ptr<float>(state),
                       (int)(phase % 3), cur_stream());
  return y;
}

// Quantise many bf16 segments of `x` into `y` (uint8/e4m3 buffer) in one launch, each under its own
// delayed-scaling state row of `states` [nseg, 4].  seg: int64 [nseg, 4] = (x offset, y offset, n8,
// first block); `blocks` = total blocks (last segment's first block + its block count).
void fp8_quant_delayed_multi(Tensor x, Tensor y, Tensor seg, Tensor states, int64_t blocks, int64_t phase) {
  check(x, BF16, "x"); check(states, F32, "states");
  TORCH_CHECK(y.device() == x.device() && y.is_contiguous() && y.element_size() == 1, "fp8_quant_delayed_multi: y");
  TORCH_CHECK(seg.device() == x.device() && seg.scalar_type() == at::kLong && seg.is_contiguous() && seg.dim() == 2 &&
                  seg.size(1) == 4 && states.numel() == seg.size(0) * 4,
              "fp8_quant_delayed_multi: seg int64 [n,4] / states f32 [n,4]");
  c10::DeviceGuard g(x.device());
  hq_fp8_quant_delayed_multi(ptr<uint16_t>(x), reinterpret_cast<uint8_t*>(y.data_ptr()), reinterpret_cast<const long long*>(seg.data_ptr<int64_t>()),
                             (int)seg.size(0), blocks, ptr<float>(states), (int)(phase % 3), cur_stream());
}

int64_t fp8_quant_multi_blocks(int64_t n8) { return hq_fp8_quant_multi_blocks(n8); }

void transpose_tiles(Tensor src, Tensor dst, Tensor tiles) {
  check(src, BF16, "src"); check(dst, BF16, "dst");
  TORCH_CHECK(tiles.device().is_cuda() && tiles.scalar_type() == at::kInt && tiles.is_contiguous() && tiles.dim() == 2 &&
              tiles.size(1) == 6, "tiles must be a contiguous int32 [n,6] GPU tensor");
  c10::DeviceGuard g(src.device());
  hq_transpose_tiles(ptr<uint16_t>(src), ptr<uint16_t>(dst), ptr<int>(tiles), (int)tiles.size(0), cur_stream());
}

// fp8 weights (1-byte elements): the e4m3 Wᵀ copies for the fp8 dgrad GEMMs
void transpose_tiles8(Tensor src, Tensor dst, Tensor tiles) {
  TORCH_CHECK(src.is_cuda() && dst.is_cuda() && src.element_size() == 1 && dst.element_size() == 1 && src.is_contiguous() &&
              dst.is_contiguous(), "transpose_tiles8: contiguous 1-byte GPU tensors");
  TORCH_CHECK(tiles.device().is_cuda() && tiles.scalar_type() == at::kInt && tiles.is_contiguous() && tiles.dim() == 2 &&
              tiles.size(1) == 6, "tiles must be a contiguous int32 [n,6] GPU tensor");
  c10::DeviceGuard g(src.device());
  hq_transpose_tiles8(reinterpret_cast<const uint8_t*>(src.data_ptr()), reinterpret_cast<uint8_t*>(dst.data_ptr()),
                      ptr<int>(tiles), (int)tiles.size(0), cur_stream());
}

// out (+)= Σ_rows part.  `part` is scratch: the two-pass reduction overwrites some of its rows.
void colsum_into(Tensor part, Tensor out, bool accumulate) {
  check(part, F32, "part"); check(out, F32, "out");
  TORCH_CHECK(part.dim() == 2 && part.size(1) == out.numel(), "colsum_into: part [P,N] / out [N]");
  c10::DeviceGuard g(part.device());
  hq_colsum(ptr<float>(part), (int)part.size(0), (int)part.size(1), ptr<float>(out), accumulate, cur_stream());
}

// x (bf16, numel % 8 == 0) -> (x8 float8_e4m3fn, scale f32[1]) with x ≈ x8 · scale (current scaling)
std::vector<Tensor> fp8_quantize(Tensor x) {
  check(x, BF16, "x");
  TORCH_CHECK(x.numel() % 8 == 0, "fp8_quantize: numel must be a multiple of 8");
  c10::DeviceGuard g(x.device());
  auto y = at::empty(x.sizes(), x.options().dtype(at::kFloat8_e4m3fn));
  auto amax = at::empty({1}, x.options().dtype(at::kInt));
  auto scale = at::empty({1}, x.options().dtype(F32));
  hq_amax_bf16(ptr<uint16_t>(x), x.numel(), ptr<unsigned>(amax), cur_stream());
  hq_fp8_quant(ptr<uint16_t>(x), ptr<uint8_t>(y), x.numel(), ptr<unsigned>(amax), ptr<float>(scale), cur_stream());
  return {y, scale.squeeze(0)};
}

// QA span head: logits [T,2] fp32 = seq[T,H] (bf16) · w[2,H]^T + b
Tensor span_fwd(Tensor seq, Tensor w, Tensor b) {
  check(seq, BF16, "seq"); check(w, F32, "w"); check(b, F32, "b");
  const int64_t H = seq.size(-1), T = seq.numel() / H;
  TORCH_CHECK(w.numel() == 2 * H && b.numel() == 2, "span_fwd: w [2,H], b [2]");
  TORCH_CHECK(H % 4 == 0 && H <= 2048, "span_fwd: hidden size");
  c10::DeviceGuard g(seq.device());
  auto logits = at::empty({T, 2}, w.options());
  hq_span_fwd(ptr<uint16_t>(seq), ptr<float>(w), ptr<float>(b), ptr<float>(logits), (int)T, (int)H, cur_stream());
  return logits;
}

// returns dseq (bf16, seq's shape); dw [2,H] f32 written (or accumulated)
Tensor span_bwd(Tensor seq, Tensor w, Tensor glog, Tensor dw, bool accumulate) {
  check(seq, BF16, "seq"); check(w, F32, "w"); check(glog, F32, "grad_logits"); check(dw, F32, "dw");
  const int64_t H = seq.size(-1), T = seq.numel() / H;
  TORCH_CHECK(w.numel() == 2 * H && dw.numel() == 2 * H && glog.numel() == 2 * T, "span_bwd: shapes");
  c10::DeviceGuard g(seq.device());
  auto dseq = at::empty_like(seq);
  auto part = at::empty({(int64_t)hq_ln_bwd_partials((int)T), 2 * H}, w.options());
  hq_span_bwd(ptr<uint16_t>(seq), ptr<float>(w), ptr<float>(glog), ptr<uint16_t>(dseq), ptr<float>(part), ptr<float>(dw),
              (int)T, (int)H, accumulate, cur_stream());
  return dseq;
}

Tensor gelu_fwd(Tensor pre) {
  check(pre, BF16, "pre");
  TORCH_CHECK(pre.numel() % 8 == 0, "numel must be a multiple of 8");
  c10::DeviceGuard g(pre.device());
  auto out = at::empty_like(pre);
  hq_gelu_fwd(ptr<uint16_t>(pre), ptr<uint16_t>(out), pre.numel(), cur_stream());
  return out;
}

Tensor gelu_bwd(Tensor dout, Tensor pre, c10::optional<Tensor> g_bias, bool accumulate) {
  check(dout, BF16, "dout"); check(pre, BF16, "pre"); check_opt(g_bias, F32, "g_bias");
  TORCH_CHECK(dout.sizes() == pre.sizes() && dout.dim() == 2, "shape");
  const int64_t T = dout.size(0), N = dout.size(1);
  TORCH_CHECK(N % 8 == 0, "N must be a multiple of 8");
  if (g_bias.has_value() && g_bias->defined()) TORCH_CHECK(g_bias->numel() == N, "g_bias shape");
  c10::DeviceGuard g(dout.device());
  auto dpre = at::empty_like(dout);
  auto part = at::empty({hq_rowblock_partials((int)T), N}, dout.options().dtype(F32));
  hq_gelu_bwd(ptr<uint16_t>(dout), ptr<uint16_t>(pre), ptr<uint16_t>(dpre), ptr<float>(part), outs4(optr<float>(g_bias)),
              (int)T, (int)N, accumulate, cur_stream());
  return dpre;
}

void bias_grad(Tensor dy, Tensor g_b, bool accumulate) {
  check(dy, BF16, "dy"); check(g_b, F32, "g_b");
  TORCH_CHECK(dy.dim() == 2 && g_b.numel() == dy.size(1) && dy.size(1) % 8 == 0, "shape");
  const int64_t T = dy.size(0), N = dy.size(1);
  c10::DeviceGuard g(dy.device());
  auto part = at::empty({hq_rowblock_partials((int)T), N}, g_b.options());
  hq_bias_grad(ptr<uint16_t>(dy), ptr<float>(part), outs4(ptr<float>(g_b)), (int)T, (int)N, accumulate, cur_stream());
}

// ------------------------------------------------------------------------------------- attention
void check_attn(const Tensor& qkv, const Tensor& kb, int64_t B, int64_t L, int64_t nh) {
  check(qkv, BF16, "qkv"); check(kb, F32, "key_bias");
  TORCH_CHECK(qkv.dim() == 2 && qkv.size(0) == B * L, "qkv rows must be B*L");
  TORCH_CHECK(qkv.size(1) % (3 * nh) == 0 && qkv.size(1) / (3 * nh) == 64, "head_dim must be 64");
  TORCH_CHECK(kb.numel() == B * L, "key_bias must be [B, L]");
  TORCH_CHECK(L >= 1 && B * nh < 65536, "grid limits");
  TORCH_CHECK(B * nh * L * L < (int64_t)std::numeric_limits<uint32_t>::max(), "B*nh*L*L exceeds 32-bit dropout index");
}

std::vector<Tensor> attn_fwd(Tensor qkv, Tensor key_bias, int64_t B, int64_t L, int64_t nh, double p, int64_t seed,
                             int64_t opid, double scale, c10::optional<Tensor> q8, int64_t phase) {
  check_attn(qkv, key_bias, B, L, nh);
  const int64_t H = qkv.size(1) / 3;
  const bool want8 = q8.has_value() && q8->defined();
  if (want8) {
    check(*q8, F32, "q8");
    TORCH_CHECK(q8->numel() == 4, "q8 must be the f32[4] delayed-scaling state");
  }
  c10::DeviceGuard g(qkv.device());
  auto ctx = at::empty({B * L, H}, qkv.options());
  auto lse = at::empty({B, nh, L}, key_bias.options());
  const int64_t mbytes = p > 0 ? (int64_t)hq_attn_mask_bytes((int)B, (int)L, (int)nh) : 0;
  auto mbits = at::empty({mbytes / 2}, qkv.options().dtype(at::kShort));
  Tensor ctx8 = want8 ? at::empty({B * L, H}, qkv.options().dtype(at::kFloat8_e4m3fn)) : Tensor();
  hq_attn_fwd(ptr<uint16_t>(qkv), ptr<float>(key_bias), ptr<uint16_t>(ctx), ptr<float>(lse),
              mbytes ? ptr<uint16_t>(mbits) : nullptr, (int)B, (int)L, (int)nh, 64, (float)p, u32(seed), u32(opid),
              (float)scale, cur_stream(), want8 ? reinterpret_cast<uint8_t*>(ctx8.data_ptr()) : nullptr,
              want8 ? ptr<float>(*q8) : nullptr, (int)(phase % 3));
  if (want8) return {ctx, lse, mbits, ctx8};
  return {ctx, lse, mbits};
}

// q8 given (--precision fp8): also dQKV as e5m2 under that delayed-scaling state -> [dqkv, dqkv8]; with
// write_bf16 = false: [empty, dqkv8, bpart] — no bf16 dQKV, the QKV bias-gradient column partials
// bpart [B·ceil(L/32), 3H] instead (colsum_into reduces them)
std::vector<Tensor> attn_bwd_impl(Tensor dctx, Tensor qkv, Tensor ctx, Tensor lse, Tensor key_bias, Tensor mbits, int64_t B,
                                  int64_t L, int64_t nh, double p, double scale, bool deterministic,
                                  c10::optional<Tensor> q8, int64_t phase, bool write_bf16 = true) {
  check_attn(qkv, key_bias, B, L, nh);
  check(dctx, BF16, "dctx"); check(ctx, BF16, "ctx"); check(lse, F32, "lse");
  const int64_t H = qkv.size(1) / 3;
  TORCH_CHECK(dctx.size(0) == B * L && dctx.size(1) == H && ctx.sizes() == dctx.sizes(), "ctx shapes");
  TORCH_CHECK(lse.numel() == B * nh * L, "lse shape");
  if (p > 0) {
    check(mbits, at::kShort, "mbits");
    TORCH_CHECK(mbits.numel() * 2 == (int64_t)hq_attn_mask_bytes((int)B, (int)L, (int)nh), "dropout mask size");
  }
  c10::DeviceGuard g(qkv.device());
  const bool want8 = q8.has_value() && q8->defined();
  TORCH_CHECK(write_bf16 || want8, "attn_bwd: write_bf16=False needs q8");
  auto dqkv = write_bf16 ? at::empty_like(qkv) : at::empty({0}, qkv.options());
  auto delta = at::empty({B, nh, L}, lse.options());
  Tensor bpart = write_bf16 ? Tensor() : at::empty({B * ((L + 31) / 32), qkv.size(1)}, lse.options());
  Tensor dqkv8;
  if (want8) {
    check(*q8, F32, "q8");
    TORCH_CHECK(q8->numel() == 4, "attn_bwd: q8 must be f32[4]");
    dqkv8 = at::empty(qkv.sizes(), qkv.options().dtype(at::kFloat8_e5m2));
  }
  hq_attn_bwd(ptr<uint16_t>(dctx), ptr<uint16_t>(qkv), ptr<uint16_t>(ctx), ptr<float>(lse), ptr<float>(key_bias),
              p > 0 ? ptr<uint16_t>(mbits) : nullptr, write_bf16 ? ptr<uint16_t>(dqkv) : nullptr, ptr<float>(delta), (int)B,
              (int)L, (int)nh, 64, (float)p, (float)scale, deterministic, cur_stream(),
              want8 ? reinterpret_cast<uint8_t*>(dqkv8.data_ptr()) : nullptr, want8 ? ptr<float>(*q8) : nullptr,
              (int)(phase % 3), write_bf16 ? nullptr : ptr<float>(bpart));
  if (!write_bf16) return {dqkv, dqkv8, bpart};
  if (want8) return {dqkv, dqkv8};
  return {dqkv};
}

Tensor attn_bwd(Tensor dctx, Tensor qkv, Tensor ctx, Tensor lse, Tensor key_bias, Tensor mbits, int64_t B, int64_t L,
                int64_t nh, double p, double scale, bool deterministic) {
  return attn_bwd_impl(dctx, qkv, ctx, lse, key_bias, mbits, B, L, nh, p, scale, deterministic, c10::nullopt, 0)[0];
}

// ------------------------------------------------------------------------------------ optimizer
std::vector<Tensor> grad_norm(Tensor grad, double max_norm) {
  check(grad, F32, "grad");
  c10::DeviceGuard g(grad.device());
  const int nparts = 1024;
  auto part = at::empty({nparts}, grad.options());
  auto norm = at::empty({1}, grad.options());
  auto coef = at::empty({1}, grad.options());
  auto s = cur_stream();
  hq_sq_norm_partials(ptr<float>(grad), grad.numel(), ptr<float>(part), nparts, s);
  hq_clip_coef(ptr<float>(part), nparts, (float)max_norm, ptr<float>(norm), ptr<float>(coef), s);
  return {norm, coef};
}

// grad norm over the chunk table (ParamStore.norm_chunks): partials[c0:c1] on the current stream
void sq_norm_chunks(Tensor grad, Tensor chunks, int64_t c0, int64_t c1, Tensor partials) {
  check(grad, F32, "grad"); check(chunks, I64, "chunks"); check(partials, F32, "partials");
  TORCH_CHECK(chunks.dim() == 2 && chunks.size(1) == 2 && partials.numel() == chunks.size(0), "chunk table / partials");
  TORCH_CHECK(0 <= c0 && c0 <= c1 && c1 <= chunks.size(0), "chunk range");
  c10::DeviceGuard g(grad.device());
  hq_sq_norm_chunks(ptr<float>(grad), ptr<int64_t>(chunks), (int)c0, (int)c1, ptr<float>(partials), cur_stream());
}

// (norm, coef) from a complete partials vector (deterministic fixed-order sum)
std::vector<Tensor> clip_from_partials(Tensor partials, double max_norm) {
  check(partials, F32, "partials");
  c10::DeviceGuard g(partials.device());
  auto norm = at::empty({1}, partials.options());
  auto coef = at::empty({1}, partials.options());
  hq_clip_coef(ptr<float>(partials), (int)partials.numel(), (float)max_norm, ptr<float>(norm), ptr<float>(coef),
               cur_stream());
  return {norm, coef};
}

HqOptGroups groups_of(const std::vector<double>& lr, const std::vector<double>& wd) {
  TORCH_CHECK(lr.size() == wd.size() && lr.size() <= (size_t)kOptMaxGroups, "at most 8 param groups");
  HqOptGroups gr{};
  for (size_t i = 0; i < lr.size(); ++i) { gr.lr[i] = (float)lr[i]; gr.wd[i] = (float)wd[i]; }
  return gr;
}

void adamw(Tensor master, c10::optional<Tensor> compute, Tensor grad, Tensor m, Tensor v, Tensor chunks,
           std::vector<double> lr, std::vector<double> wd, double beta1, double beta2, double eps, double step_mult,
           c10::optional<Tensor> clip_coef) {
  check(master, F32, "master"); check_opt(compute, BF16, "compute"); check(grad, F32, "grad");
  check(m, F32, "exp_avg"); check(v, F32, "exp_avg_sq"); check(chunks, I64, "chunks"); check_opt(clip_coef, F32, "clip");
  TORCH_CHECK(grad.numel() == master.numel() && m.numel() == master.numel() && v.numel() == master.numel(), "arena sizes");
  if (compute.has_value() && compute->defined()) TORCH_CHECK(compute->numel() == master.numel(), "compute size");
  TORCH_CHECK(chunks.dim() == 2 && chunks.size(1) == 2, "chunks must be [n,2] int64");
  c10::DeviceGuard g(master.device());
  hq_adamw(ptr<float>(master), optr<uint16_t>(compute), ptr<float>(grad), ptr<float>(m), ptr<float>(v),
           reinterpret_cast<const HqOptChunk*>(chunks.data_ptr()), (int)chunks.size(0), groups_of(lr, wd), (float)beta1,
           (float)beta2, (float)eps, (float)step_mult, optr<float>(clip_coef), cur_stream());
}

void adamod(Tensor master, c10::optional<Tensor> compute, Tensor grad, Tensor m, Tensor v, Tensor n, Tensor chunks,
            std::vector<double> lr, std::vector<double> wd, double beta1, double beta2, double beta3, double eps,
            double bias_corr, c10::optional<Tensor> clip_coef) {
  check(master, F32, "master"); check_opt(compute, BF16, "compute"); check(grad, F32, "grad");
  check(m, F32, "exp_avg"); check(v, F32, "exp_avg_sq"); check(n, F32, "exp_avg_lr"); check(chunks, I64, "chunks");
  check_opt(clip_coef, F32, "clip");
  TORCH_CHECK(grad.numel() == master.numel() && m.numel() == master.numel() && v.numel() == master.numel() &&
                  n.numel() == master.numel(), "arena sizes");
  c10::DeviceGuard g(master.device());
  hq_adamod(ptr<float>(master), optr<uint16_t>(compute), ptr<float>(grad), ptr<float>(m), ptr<float>(v), ptr<float>(n),
            reinterpret_cast<const HqOptChunk*>(chunks.data_ptr()), (int)chunks.size(0), groups_of(lr, wd), (float)beta1,
            (float)beta2, (float)beta3, (float)eps, (float)bias_corr, optr<float>(clip_coef), cur_stream());
}

void cast_f32_bf16(Tensor src, Tensor dst, double scale) {
  check(src, F32, "src"); check(dst, BF16, "dst");
  TORCH_CHECK(src.numel() == dst.numel(), "size");
  c10::DeviceGuard g(src.device());
  hq_cast_f32_bf16(ptr<float>(src), ptr<uint16_t>(dst), src.numel(), (float)scale, cur_stream());
}

// ------------------------------------------------------------------------ fused QA heads + losses
// Ticket words of the in-launch hand-offs (heads.hip), one zeroed int32[4] per (device, stream): [0] fwd,
// [1] loss.  The last-arriving block resets its word, so a buffer is zeroed exactly once.
unsigned* ticket(const Tensor& like, int slot) {
  static std::map<std::pair<int, hipStream_t>, Tensor> words;
  const auto key = std::make_pair((int)like.get_device(), cur_stream());
  auto it = words.find(key);
  if (it == words.end()) it = words.emplace(key, at::zeros({4}, like.options().dtype(at::kInt))).first;
  return reinterpret_cast<unsigned*>(it->second.data_ptr<int>()) + slot;
}

HqHeadWeights head_weights(const std::vector<Tensor>& w, int64_t H, int64_t NL) {
  TORCH_CHECK(w.size() == 10, "head weights: wp, bp, wc, bc, wrs, brs, wre, bre, wsp, bsp");
  const int64_t numel[10] = {H * H, H, NL * H, NL, H, 1, H, 1, 2 * H, 2};
  for (int i = 0; i < 10; ++i) {
    check(w[i], F32, "head weight");
    TORCH_CHECK(w[i].numel() == numel[i], "head weight ", i, ": ", w[i].numel(), " elements, expected ", numel[i]);
  }
  return HqHeadWeights{ptr<float>(w[0]), ptr<float>(w[1]), ptr<float>(w[2]), ptr<float>(w[3]), ptr<float>(w[4]),
                       ptr<float>(w[5]), ptr<float>(w[6]), ptr<float>(w[7]), ptr<float>(w[8]), ptr<float>(w[9])};
}

void check_heads_shape(const Tensor& seq, int64_t L, int64_t NL) {
  TORCH_CHECK(seq.is_cuda() && seq.is_contiguous() && (seq.scalar_type() == BF16 || seq.scalar_type() == F32),
              "seq must be a contiguous bf16 or fp32 GPU tensor");
  const int64_t H = seq.size(-1), T = seq.numel() / H;
  TORCH_CHECK(L > 0 && T % L == 0, "seq rows must be B*L");
  TORCH_CHECK(H % 64 == 0 && H <= 2048, "fused heads need hidden % 64 == 0 and <= 2048, got ", H);
  TORCH_CHECK(NL >= 1 && NL <= 8, "fused heads support 1..8 classes, got ", NL);
  TORCH_CHECK(T * H < (int64_t)std::numeric_limits<int32_t>::max(), "T*H exceeds 32-bit indexing");
}

// returns logits [T,2], pooled [B,H], cls [B,NL], reg [B,2] (sigmoid outputs)
std::vector<Tensor> qa_heads_fwd(Tensor seq, int64_t L, std::vector<Tensor> w, double p, int64_t seed, int64_t opid) {
  const int64_t H = seq.size(-1), NL = w.size() > 3 ? w[3].numel() : 0;
  check_heads_shape(seq, L, NL);
  const int64_t T = seq.numel() / H, B = T / L;
  const HqHeadWeights hw = head_weights(w, H, NL);
  c10::DeviceGuard g(seq.device());
  auto f = w[0].options();
  auto logits = at::empty({T, 2}, f);
  auto pooled = at::empty({B, H}, f);
  auto cls = at::empty({B, NL}, f);
  auto reg = at::empty({B, 2}, f);
  auto hpart = at::empty({(int64_t)hq_qa_heads_fwd_scratch((int)B, (int)H)}, f);
  hq_qa_heads_fwd(seq.data_ptr(), hw, ptr<float>(logits), ptr<float>(pooled), ptr<float>(cls), ptr<float>(reg),
                  ptr<float>(hpart), ticket(seq, 0), (int)B, (int)L, (int)H, (int)NL, (float)p, u32(seed), u32(opid),
                  cur_stream(), seq.scalar_type() == F32);
  return {logits, pooled, cls, reg};
}

// returns losses [6], dlog [T,2], dheads [B,16]
std::vector<Tensor> qa_loss(Tensor logits, Tensor cls, Tensor reg, Tensor t_start, Tensor t_end, Tensor t_rs, Tensor t_re,
                            Tensor t_cls, c10::optional<Tensor> lw, int64_t kind, int64_t ignore_cls,
                            std::vector<double> weights, double alpha, double gamma, double conf, double fill,
                            c10::optional<Tensor> seg_len) {
  check(logits, F32, "logits"); check(cls, F32, "cls"); check(reg, F32, "reg");
  check(t_start, I64, "start_class"); check(t_end, I64, "end_class"); check(t_cls, I64, "cls target");
  check(t_rs, F32, "start_reg"); check(t_re, F32, "end_reg"); check_opt(lw, F32, "label_weights");
  const int64_t B = cls.size(0), NL = cls.size(1), T = logits.size(0);
  TORCH_CHECK(logits.dim() == 2 && logits.size(1) == 2 && B > 0 && T % B == 0, "logits [B*L, 2]");
  TORCH_CHECK(NL >= 1 && NL <= 8 && reg.numel() == 2 * B, "cls [B, NL<=8], reg [B, 2]");
  TORCH_CHECK(t_start.numel() == B && t_end.numel() == B && t_cls.numel() == B && t_rs.numel() == B &&
                  t_re.numel() == B, "targets must have B elements");
  TORCH_CHECK(!lw.has_value() || !lw->defined() || lw->numel() == NL, "label weights [NL]");
  TORCH_CHECK(weights.size() == 5 && kind >= 0 && kind <= 2, "loss config");
  int nseg = 1;
  if (seg_len.has_value() && seg_len->defined()) {   // exact-objective merge: one segment per micro-batch
    check(*seg_len, at::kInt, "segment lengths");
    nseg = (int)seg_len->numel();
    TORCH_CHECK(nseg >= 1 && B % nseg == 0, "segments must split the batch into equal parts");
  }
  c10::DeviceGuard g(logits.device());
  auto f = logits.options();
  auto losses = at::empty({6}, f);
  auto dlog = at::empty({T, 2}, f);
  auto dheads = at::empty({B, 16}, f);
  auto part = at::empty({(int64_t)hq_qa_loss_partials((int)B), 4}, f);
  HqLossCfg cfg;
  cfg.kind = (int)kind;
  cfg.ignore_cls = (int)ignore_cls;
  for (int i = 0; i < 5; ++i) cfg.w[i] = (float)weights[i];
  cfg.alpha = (float)alpha; cfg.gamma = (float)gamma; cfg.conf = (float)conf; cfg.fill = (float)fill;
  hq_qa_loss(ptr<float>(logits), ptr<float>(cls), ptr<float>(reg), ptr<int64_t>(t_start), ptr<int64_t>(t_end),
             ptr<int64_t>(t_cls), ptr<float>(t_rs), ptr<float>(t_re), optr<float>(lw), ptr<float>(dlog), ptr<float>(dheads),
             ptr<float>(losses), ptr<float>(part), ticket(logits, 1), (int)B, (int)(T / B), (int)NL, cfg,
             nseg > 1 || (seg_len.has_value() && seg_len->defined()) ? optr<int>(seg_len) : nullptr, nseg, cur_stream());
  return {losses, dlog, dheads};
}

// writes the 10 head gradients (wp, bp, wc, bc, wrs, brs, wre, bre, wsp, bsp) (+)=; returns dseq (bf16, seq's shape)
Tensor qa_heads_bwd(Tensor seq, int64_t L, Tensor dlog, Tensor dheads, c10::optional<Tensor> gscale, Tensor pooled,
                    Tensor reg, std::vector<Tensor> w, std::vector<Tensor> grads, bool accumulate, double p, int64_t seed,
                    int64_t opid) {
  const int64_t H = seq.size(-1), NL = w.size() > 3 ? w[3].numel() : 0;
  check_heads_shape(seq, L, NL);
  const int64_t T = seq.numel() / H, B = T / L;
  check(dlog, F32, "dlog"); check(dheads, F32, "dheads"); check(pooled, F32, "pooled"); check(reg, F32, "reg");
  check_opt(gscale, F32, "gscale");
  TORCH_CHECK(dlog.numel() == 2 * T && dheads.numel() == 16 * B && pooled.numel() == B * H && reg.numel() == 2 * B,
              "qa_heads_bwd: operand shapes");
  TORCH_CHECK(!gscale.has_value() || !gscale->defined() || gscale->numel() == 1, "gscale is a scalar");
  const HqHeadWeights hw = head_weights(w, H, NL);
  const HqHeadWeights hg = head_weights(grads, H, NL);  // same shapes / dtype checks for the gradients
  HqHeadGrads gg{const_cast<float*>(hg.wp), const_cast<float*>(hg.bp), const_cast<float*>(hg.wc),
                 const_cast<float*>(hg.bc), const_cast<float*>(hg.wrs), const_cast<float*>(hg.brs),
                 const_cast<float*>(hg.wre), const_cast<float*>(hg.bre), const_cast<float*>(hg.wsp),
                 const_cast<float*>(hg.bsp)};
  c10::DeviceGuard g(seq.device());
  auto dseq = at::empty_like(seq);
  auto part = at::empty({(int64_t)hq_qa_heads_bwd_span_blocks((int)T), 2 * H + 2}, pooled.options());
  auto dpre = at::empty({B, H}, pooled.options());
  hq_qa_heads_bwd(seq.data_ptr(), ptr<float>(dlog), ptr<float>(dheads), optr<float>(gscale), ptr<float>(pooled),
                  ptr<float>(reg), hw, gg, dseq.data_ptr(), ptr<float>(part), (int)B, (int)L, (int)H, (int)NL,
                  accumulate, (float)p, u32(seed), u32(opid), cur_stream(), seq.scalar_type() == F32, ptr<float>(dpre));
  return dseq;
}

}  // namespace

// ---------------------------------------------------------------- --precision fp32 (f32_ops.hip)
static void f32_rows(const Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == F32 && t.is_contiguous(), n, " must be a contiguous fp32 GPU tensor");
}

std::vector<Tensor> f32_embed_fwd(Tensor ids, Tensor pids, Tensor tids, Tensor ww, Tensor wp, Tensor wt, Tensor gamma,
                                  Tensor beta, double eps, double p, int64_t seed, int64_t opid) {
  check(ids, I64, "ids"); check(pids, I64, "pos_ids"); check(tids, I64, "type_ids");
  f32_rows(ww, "w_word"); f32_rows(wp, "w_pos"); f32_rows(wt, "w_type"); f32_rows(gamma, "gamma"); f32_rows(beta, "beta");
  const int64_t T = ids.numel(), H = ww.size(1);
  TORCH_CHECK(pids.numel() == T && tids.numel() == T && wp.size(1) == H && wt.size(1) == H && gamma.numel() == H, "shapes");
  c10::DeviceGuard g(ww.device());
  auto y = at::empty({T, H}, ww.options());
  auto mean = at::empty({T}, ww.options());
  auto rstd = at::empty({T}, ww.options());
  hq_f32_embed_fwd(ptr<int64_t>(ids), ptr<int64_t>(pids), ptr<int64_t>(tids), ptr<float>(ww), ptr<float>(wp), ptr<float>(wt),
                   ptr<float>(gamma), ptr<float>(beta), ptr<float>(y), ptr<float>(mean), ptr<float>(rstd), (int)T, (int)H,
                   (float)eps, (float)p, u32(seed), u32(opid), (int)ww.size(0), (int)wp.size(0), (int)wt.size(0),
                   cur_stream());
  return {y, mean, rstd};
}

void f32_embed_bwd(Tensor dy, Tensor ids, Tensor pids, Tensor tids, Tensor ww, Tensor wp, Tensor wt, Tensor gamma, Tensor mean,
                   Tensor rstd, double p, int64_t seed, int64_t opid, Tensor g_word, Tensor g_pos, Tensor g_type,
                   Tensor g_gamma, Tensor g_beta, bool accumulate, int64_t pad_word, int64_t pad_pos) {
  check(ids, I64, "ids"); check(pids, I64, "pos_ids"); check(tids, I64, "type_ids");
  for (auto* t : {&dy, &ww, &wp, &wt, &gamma, &mean, &rstd, &g_word, &g_pos, &g_type, &g_gamma, &g_beta}) f32_rows(*t, "f32 operand");
  const int64_t T = ids.numel(), H = ww.size(1);
  TORCH_CHECK(dy.size(0) == T && dy.size(1) == H, "dy shape");
  TORCH_CHECK(g_word.sizes() == ww.sizes() && g_pos.sizes() == wp.sizes() && g_type.sizes() == wt.sizes(), "grad shapes");
  c10::DeviceGuard g(dy.device());
  auto s = cur_stream();
  const int n_types = (int)wt.size(0);
  if (!accumulate) {
    hq_zero_f32(ptr<float>(g_word), (size_t)g_word.numel(), s);
    hq_zero_f32(ptr<float>(g_pos), (size_t)g_pos.numel(), s);
    if (n_types > 2) hq_zero_f32(ptr<float>(g_type), (size_t)g_type.numel(), s);   // else folded from partials
  }
  auto part = at::empty({hq_f32_part_rows((int)T), 4 * H}, dy.options());
  float* t0 = ptr<float>(g_type);
  hq_f32_embed_bwd(ptr<float>(dy), ptr<int64_t>(ids), ptr<int64_t>(pids), ptr<int64_t>(tids), ptr<float>(ww), ptr<float>(wp),
                   ptr<float>(wt), ptr<float>(gamma), ptr<float>(mean), ptr<float>(rstd), ptr<float>(g_word),
                   ptr<float>(g_pos), t0, ptr<float>(part),
                   outs4(ptr<float>(g_gamma), ptr<float>(g_beta), n_types <= 2 ? t0 : nullptr, n_types == 2 ? t0 + H : nullptr),
                   (int)T, (int)H, (int)pad_word, (int)pad_pos, (float)p, u32(seed), u32(opid), accumulate,
                   (int)ww.size(0), (int)wp.size(0), (int)wt.size(0), s);
}

std::vector<Tensor> f32_ln_fwd(Tensor a, Tensor resid, Tensor gamma, Tensor beta, double eps, double p, int64_t seed,
                               int64_t opid) {
  f32_rows(a, "a"); f32_rows(resid, "resid"); f32_rows(gamma, "gamma"); f32_rows(beta, "beta");
  TORCH_CHECK(a.dim() == 2 && a.sizes() == resid.sizes() && gamma.numel() == a.size(1), "ln shapes");
  c10::DeviceGuard g(a.device());
  const int64_t T = a.size(0), H = a.size(1);
  auto y = at::empty_like(a), z = at::empty_like(a);
  auto mean = at::empty({T}, a.options()), rstd = at::empty({T}, a.options());
  hq_f32_ln_fwd(ptr<float>(a), ptr<float>(resid), ptr<float>(gamma), ptr<float>(beta), ptr<float>(y), ptr<float>(z),
                ptr<float>(mean), ptr<float>(rstd), (int)T, (int)H, (float)eps, (float)p, u32(seed), u32(opid), cur_stream());
  return {y, z, mean, rstd};
}

std::vector<Tensor> f32_ln_bwd(Tensor dy, c10::optional<Tensor> dy2, Tensor z, Tensor gamma, Tensor mean, Tensor rstd,
                               double p, int64_t seed, int64_t opid, c10::optional<Tensor> g_gamma,
                               c10::optional<Tensor> g_beta, c10::optional<Tensor> g_bias, bool accumulate,
                               c10::optional<Tensor> beta) {
  f32_rows(dy, "dy"); f32_rows(z, "z"); f32_rows(gamma, "gamma"); f32_rows(mean, "mean"); f32_rows(rstd, "rstd");
  if (dy2.has_value() && dy2->defined()) { f32_rows(*dy2, "dy2"); TORCH_CHECK(dy2->sizes() == dy.sizes(), "dy2 shape"); }
  if (beta.has_value() && beta->defined()) f32_rows(*beta, "beta");
  TORCH_CHECK(dy.sizes() == z.sizes() && gamma.numel() == dy.size(1), "ln_bwd shapes");
  c10::DeviceGuard g(dy.device());
  const int64_t T = dy.size(0), H = dy.size(1);
  auto dz = at::empty_like(dy), da = at::empty_like(dy);
  auto part = at::empty({hq_f32_part_rows((int)T), 3 * H}, dy.options());
  hq_f32_ln_bwd(ptr<float>(dy), optr<float>(dy2), ptr<float>(z), ptr<float>(gamma), optr<float>(beta), ptr<float>(mean),
                ptr<float>(rstd), ptr<float>(dz), ptr<float>(da), ptr<float>(part),
                outs4(optr<float>(g_gamma), optr<float>(g_beta), optr<float>(g_bias)), (int)T, (int)H, (float)p, u32(seed),
                u32(opid), accumulate, cur_stream());
  return {dz, da};
}

Tensor f32_gelu_fwd(Tensor x) {
  f32_rows(x, "x");
  c10::DeviceGuard g(x.device());
  auto y = at::empty_like(x);
  hq_f32_gelu_fwd(ptr<float>(x), ptr<float>(y), x.numel(), cur_stream());
  return y;
}

Tensor f32_gelu_bwd(Tensor dout, Tensor x, c10::optional<Tensor> g_bias, bool accumulate) {
  f32_rows(dout, "dout"); f32_rows(x, "pre");
  TORCH_CHECK(dout.sizes() == x.sizes() && dout.dim() == 2, "gelu_bwd shapes");
  c10::DeviceGuard g(x.device());
  const int64_t T = x.size(0), N = x.size(1);
  auto d = at::empty_like(x);
  auto part = at::empty({hq_f32_part_rows((int)T), N}, x.options());
  hq_f32_gelu_bwd(ptr<float>(dout), ptr<float>(x), ptr<float>(d), ptr<float>(part), optr<float>(g_bias), (int)T, (int)N,
                  accumulate, cur_stream());
  return d;
}

void f32_colsum(Tensor x, Tensor out, bool accumulate) {
  f32_rows(x, "x"); f32_rows(out, "out");
  TORCH_CHECK(x.dim() == 2 && out.numel() == x.size(1), "colsum shapes");
  c10::DeviceGuard g(x.device());
  auto part = at::empty({hq_f32_part_rows((int)x.size(0)), x.size(1)}, x.options());
  hq_f32_colsum(ptr<float>(x), ptr<float>(part), ptr<float>(out), (int)x.size(0), (int)x.size(1), accumulate, cur_stream());
}

std::vector<Tensor> f32_attn_fwd(Tensor qkv, Tensor key_bias, int64_t B, int64_t L, int64_t nh, double p, int64_t seed,
                                 int64_t opid, double scale) {
  f32_rows(qkv, "qkv"); f32_rows(key_bias, "key_bias");
  TORCH_CHECK(qkv.size(0) == B * L && qkv.size(1) == 3 * nh * 64 && key_bias.numel() == B * L, "f32 attention: head_dim 64");
  TORCH_CHECK(B * nh * L * L < (int64_t(1) << 32), "f32 attention: dropout element index must fit 32 bits");
  c10::DeviceGuard g(qkv.device());
  auto ctx = at::empty({B * L, nh * 64}, qkv.options());
  auto lse = at::empty({B, nh, L}, qkv.options());
  hq_f32_attn_fwd(ptr<float>(qkv), ptr<float>(key_bias), ptr<float>(ctx), ptr<float>(lse), (int)B, (int)L, (int)nh, (float)p,
                  u32(seed), u32(opid), (float)scale, cur_stream());
  return {ctx, lse};
}

Tensor f32_attn_bwd(Tensor dctx, Tensor qkv, Tensor ctx, Tensor lse, Tensor key_bias, int64_t B, int64_t L, int64_t nh,
                    double p, int64_t seed, int64_t opid, double scale) {
  f32_rows(dctx, "dctx"); f32_rows(qkv, "qkv"); f32_rows(ctx, "ctx"); f32_rows(lse, "lse"); f32_rows(key_bias, "key_bias");
  TORCH_CHECK(qkv.size(0) == B * L && qkv.size(1) == 3 * nh * 64 && dctx.sizes() == ctx.sizes() &&
              ctx.size(0) == B * L && ctx.size(1) == nh * 64 && lse.numel() == B * nh * L && key_bias.numel() == B * L,
              "f32 attention backward shapes");
  c10::DeviceGuard g(qkv.device());
  auto dqkv = at::empty_like(qkv);
  auto delta = at::empty({B, nh, L}, qkv.options());
  hq_f32_attn_bwd(ptr<float>(dctx), ptr<float>(qkv), ptr<float>(ctx), ptr<float>(lse), ptr<float>(key_bias), ptr<float>(dqkv),
                  ptr<float>(delta), (int)B, (int)L, (int)nh, (float)p, u32(seed), u32(opid), (float)scale, cur_stream());
  return dqkv;
}

PYBIND11_MODULE(_hq_kernels, m) {
  m.doc() = "gfx950 HIP kernels + RCCL reducer for ml_recipe_distributed_pytorch_amd";
  m.def("embed_fwd", &embed_fwd);
  m.def("embed_bwd", &embed_bwd, py::arg("dy"), py::arg("ids"), py::arg("pids"), py::arg("tids"), py::arg("ww"),
        py::arg("wp"), py::arg("wt"), py::arg("gamma"), py::arg("mean"), py::arg("rstd"), py::arg("p"), py::arg("seed"),
        py::arg("opid"), py::arg("g_word"), py::arg("g_pos"), py::arg("g_type"), py::arg("g_gamma"), py::arg("g_beta"),
        py::arg("accumulate"), py::arg("pad_word"), py::arg("pad_pos"), py::arg("seq_len") = 0);
  m.def("ln_fwd", &ln_fwd, py::arg("a"), py::arg("resid"), py::arg("gamma"), py::arg("beta"), py::arg("eps"), py::arg("p"),
        py::arg("seed"), py::arg("opid"), py::arg("q8") = py::none(), py::arg("phase") = 0, py::arg("store_z") = true);
  m.def("ln_bwd", &ln_bwd, py::arg("dy"), py::arg("dy2"), py::arg("z"), py::arg("gamma"), py::arg("mean"), py::arg("rstd"),
        py::arg("p"), py::arg("seed"), py::arg("opid"), py::arg("g_gamma"), py::arg("g_beta"), py::arg("g_bias"),
        py::arg("accumulate"), py::arg("q8") = py::none(), py::arg("phase") = 0, py::arg("write_da") = true,
        py::arg("beta") = py::none());
  m.def("gelu_fwd", &gelu_fwd);
  m.def("gemm_nt", &gemm_nt, py::arg("A"), py::arg("B"), py::arg("epi"), py::arg("bias") = py::none(),
        py::arg("pre") = py::none(), py::arg("resid") = py::none(), py::arg("part") = py::none(),
        py::arg("out") = py::none(), py::arg("p") = 0.0, py::arg("seed") = 0, py::arg("opid") = 0);
  m.def("gemm_nt_supported", &gemm_nt_supported);
  m.def("gemm_nt_part_rows", [](int64_t M, int64_t N, int64_t K) {
    return (int64_t)hq_gemm_nt_part_rows((int)M, (int)N, (int)K);
  });
  m.def("gemm_set_variant", [](int64_t v) { hq_gemm_set_variant((int)v); });
  m.def("gemm_set_store_policy", [](int64_t v) { hq_gemm_set_store_policy((int)v); });
  m.def("gemm_set_stagger", [](int64_t v) { hq_gemm_set_stagger((int)v); });
  m.def("gemm_tn_set_variant", [](int64_t v) { hq_gemm_tn_set_variant((int)v); });
  m.def("gemm_set_sched", [](int64_t v) { hq_gemm_set_sched((int)v); });
  m.def("gemm_get_sched", []() { return (int64_t)hq_gemm_get_sched(); });
  m.def("gemm_tn", &gemm_tn, py::arg("dy"), py::arg("x"), py::arg("out"), py::arg("accumulate") = false,
        py::arg("splits") = 0, py::arg("bias_out") = py::none());
  m.def("gemm_tn_splits", &gemm_tn_splits);
  m.def("gemm_f32", &gemm_f32, py::arg("A"), py::arg("B"), py::arg("C"), py::arg("M"), py::arg("N"), py::arg("K"),
        py::arg("sa"), py::arg("sb"), py::arg("sc"), py::arg("batch") = 1, py::arg("nb_in") = 1, py::arg("alpha") = 1.0,
        py::arg("bias") = py::none(), py::arg("R") = py::none(), py::arg("ldr") = 0);
  m.def("attn_set_force_slow", [](int64_t v) { hq_attn_set_force_slow((int)v); });
  m.def("transpose_tiles", &transpose_tiles);
  m.def("transpose_tiles8", &transpose_tiles8);
  m.def("colsum_into", &colsum_into);
  m.def("f32_embed_fwd", &f32_embed_fwd);
  m.def("f32_embed_bwd", &f32_embed_bwd);
  m.def("f32_ln_fwd", &f32_ln_fwd);
  m.def("f32_ln_bwd", &f32_ln_bwd, py::arg("dy"), py::arg("dy2"), py::arg("z"), py::arg("gamma"), py::arg("mean"),
        py::arg("rstd"), py::arg("p"), py::arg("seed"), py::arg("opid"), py::arg("g_gamma"), py::arg("g_beta"),
        py::arg("g_bias"), py::arg("accumulate"), py::arg("beta") = py::none());
  m.def("f32_gelu_fwd", &f32_gelu_fwd);
  m.def("f32_gelu_bwd", &f32_gelu_bwd);
  m.def("f32_colsum", &f32_colsum);
  m.def("f32_attn_fwd", &f32_attn_fwd);
  m.def("f32_attn_bwd", &f32_attn_bwd);
  m.def("key_bias", [](Tensor mask) {   // bool / uint8 attention mask -> fp32 additive key bias, same shape
    TORCH_CHECK(mask.is_cuda() && mask.is_contiguous() && mask.element_size() == 1 &&
                (mask.scalar_type() == at::kBool || mask.scalar_type() == at::kByte), "key_bias: bool / uint8 GPU mask");
    c10::DeviceGuard g(mask.device());
    auto kb = at::empty(mask.sizes(), mask.options().dtype(at::kFloat));
    hq_key_bias(reinterpret_cast<const uint8_t*>(mask.data_ptr()), ptr<float>(kb), (int)mask.numel(), cur_stream());
    return kb;
  });
  m.def("ln_guard", [](Tensor master, Tensor goff, Tensor boff, int64_t H, double ratio) {
    check(master, F32, "master");
    TORCH_CHECK(goff.is_cuda() && boff.is_cuda() && goff.scalar_type() == at::kLong && boff.scalar_type() == at::kLong &&
                goff.numel() == boff.numel() && goff.is_contiguous() && boff.is_contiguous(), "ln_guard: offsets");
    // (offsets are validated against the arena on the host when the caller builds them: no device read here)
    c10::DeviceGuard g(master.device());
    auto flags = at::empty({goff.numel()}, master.options().dtype(at::kBool));
    hq_ln_guard(ptr<float>(master), goff.data_ptr<int64_t>(), boff.data_ptr<int64_t>(), (int)goff.numel(), (int)H,
                (float)ratio, reinterpret_cast<uint8_t*>(flags.data_ptr()), cur_stream());
    return flags;
  });
  m.def("sort_ids", [](Tensor ids, int64_t V) {   // the embedding backward's stable id sort (tests)
    TORCH_CHECK(ids.is_cuda() && ids.scalar_type() == at::kLong && ids.is_contiguous() && ids.dim() == 1,
                "sort_ids: ids must be a contiguous int64 GPU vector");
    c10::DeviceGuard g(ids.device());
    const int T = (int)ids.numel();
    auto buf = at::empty({4, std::max(T, 1)}, ids.options().dtype(at::kInt));
    auto hist = at::empty({(int64_t)std::max<size_t>(hq_sort_ids_bytes(T, (int)V), 4)}, ids.options().dtype(at::kByte));
    int32_t* b = buf.data_ptr<int32_t>();
    const int64_t stride = std::max(T, 1);
    hq_sort_ids(ids.data_ptr<int64_t>(), T, (int)V, b, b + stride, b + 2 * stride, b + 3 * stride, hist.data_ptr(),
                hist.numel(), cur_stream());
    return std::make_pair(buf[2].narrow(0, 0, T), buf[3].narrow(0, 0, T));
  });
  m.def("gelud_code", []() { return std::make_pair((double)kHqGdLo, (double)kHqGdStep); },
        "(lo, step) of the fp8 path's 8-bit gelu' code: g = lo + q·step");
  m.def("gelud_code_enc", []() { return std::make_pair((double)kHqGdInv, (double)kHqGdOff); },
        "(inv, off) of the encoder: q = round(fma(g, inv, off)), clamp 0..255 (fp32)");
  m.def("gelud_encode8", [](Tensor g) {
    check(g, BF16, "g");
    TORCH_CHECK(g.numel() % 8 == 0, "gelud_encode8: numel must be a multiple of 8");
    c10::DeviceGuard dg(g.device());
    auto q = at::empty(g.sizes(), g.options().dtype(at::kByte));
    hq_gelud_encode8(ptr<uint16_t>(g), q.data_ptr<uint8_t>(), g.numel(), cur_stream());
    return q;
  });
  m.def("fp8_quantize", &fp8_quantize);
  m.def("fp8_quant_delayed", &fp8_quant_delayed);
  m.def("fp8_quant_delayed_multi", &fp8_quant_delayed_multi);
  m.def("fp8_fold_defer", [](bool on) { return hq_fp8_fold_defer(on ? 1 : 0); },
        "batch the delayed-scaling amax folds of the fp8 producers until fp8_fold_flush (False: flush, immediate folds)");
  m.def("fp8_fold_flush", []() { hq_fp8_fold_flush(); });
  m.def("fp8_fold_pending", []() { return hq_fp8_fold_pending(); });
  m.def("fp8_quant_multi_blocks", &fp8_quant_multi_blocks);
  m.def("gemm_fp8_supported", &gemm_fp8_supported);
  m.def("gemm_fp8_set_variant", [](int64_t v) { hq_gemm_fp8_set_variant((int)v); });
  m.def("gemm_tn8_splits", &gemm_tn8_splits);
  m.def("gemm_tn8", &gemm_tn8);
  m.def("gemm_fp8", &gemm_fp8, py::arg("A8"), py::arg("B8"), py::arg("epi"), py::arg("bias"), py::arg("sa"), py::arg("sb"),
        py::arg("pre") = py::none(), py::arg("out8") = py::none(), py::arg("state") = py::none(), py::arg("phase") = 0,
        py::arg("part") = py::none(), py::arg("resid") = py::none(), py::arg("write_out") = true);
  m.def("span_fwd", &span_fwd);
  m.def("span_bwd", &span_bwd);
  m.def("set_dropout_seed", [](c10::optional<Tensor> t) {
    if (t.has_value() && t->defined()) {
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kInt && t->numel() >= 1, "seed must be a GPU int32 tensor");
      hq_set_dropout_seed_ptr(reinterpret_cast<const uint32_t*>(t->data_ptr()));
    } else {
      hq_set_dropout_seed_ptr(nullptr);
    }
  });
  m.def("qa_heads_fwd", &qa_heads_fwd);
  m.def("qa_loss", &qa_loss);
  m.def("qa_heads_bwd", &qa_heads_bwd);
  m.def("gelu_bwd", &gelu_bwd);
  m.def("bias_grad", &bias_grad);
  m.def("attn_fwd", &attn_fwd, py::arg("qkv"), py::arg("key_bias"), py::arg("B"), py::arg("L"), py::arg("nh"),
        py::arg("p"), py::arg("seed"), py::arg("opid"), py::arg("scale"), py::arg("q8") = py::none(),
        py::arg("phase") = 0);
  m.def("attn_bwd", &attn_bwd);
  m.def("attn_bwd_q8", [](Tensor dctx, Tensor qkv, Tensor ctx, Tensor lse, Tensor key_bias, Tensor mbits, int64_t B,
                          int64_t L, int64_t nh, double p, double scale, bool deterministic, Tensor q8, int64_t phase,
                          bool write_bf16) {
    return attn_bwd_impl(dctx, qkv, ctx, lse, key_bias, mbits, B, L, nh, p, scale, deterministic, q8, phase, write_bf16);
  }, py::arg("dctx"), py::arg("qkv"), py::arg("ctx"), py::arg("lse"), py::arg("key_bias"), py::arg("mbits"), py::arg("B"),
     py::arg("L"), py::arg("nh"), py::arg("p"), py::arg("scale"), py::arg("deterministic"), py::arg("q8"), py::arg("phase"),
     py::arg("write_bf16") = true);
  m.def("grad_norm", &grad_norm);
  m.def("sq_norm_chunks", &sq_norm_chunks);
  m.def("clip_from_partials", &clip_from_partials);
  m.def("sq_norm_partials", [](Tensor x, int64_t nparts) {
    check(x, F32, "x");
    TORCH_CHECK(x.is_contiguous(), "x must be contiguous");
    c10::DeviceGuard g(x.device());
    auto part = at::empty({nparts}, x.options());
    hq_sq_norm_partials(ptr<float>(x), x.numel(), ptr<float>(part), (int)nparts, cur_stream());
    return part;
  });
  m.def("fingerprint", [](Tensor x, int64_t nparts) {
    check(x, F32, "x");
    TORCH_CHECK(x.is_contiguous(), "x must be contiguous");
    TORCH_CHECK(nparts > 0 && nparts <= 65535, "nparts out of range");
    c10::DeviceGuard g(x.device());
    auto out = at::empty({nparts}, x.options().dtype(at::kLong));
    hq_fingerprint(ptr<float>(x), x.numel(), (int)nparts, reinterpret_cast<uint64_t*>(out.data_ptr<int64_t>()),
                   cur_stream());
    return out;
  });
  m.def("adamw", &adamw);
  m.def("adamod", &adamod);
  m.def("cast_f32_bf16", &cast_f32_bf16);
  m.def("rccl_unique_id", []() { return py::bytes(hq_rccl_unique_id()); });
  py::class_<HqReducer>(m, "Reducer")
      .def(py::init([](int rank, int world, py::bytes uid, int device) {
             return new HqReducer(rank, world, std::string(uid), device);
           }))
      .def("allreduce_f32", &HqReducer::allreduce_f32, py::arg("ptr"), py::arg("count"), py::arg("stream"),
           py::arg("op") = 0, py::call_guard<py::gil_scoped_release>())
      .def("allreduce_bf16", &HqReducer::allreduce_bf16, py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &HqReducer::broadcast, py::call_guard<py::gil_scoped_release>())
      .def("wait", &HqReducer::wait)
      .def("probe_f32", &HqReducer::probe_f32)
      .def("sq_norm_chunks", &HqReducer::sq_norm_chunks)
      .def("fence_from", &HqReducer::fence_from)
      .def("synchronize", &HqReducer::synchronize, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("comm_stream", &HqReducer::comm_stream)
      .def_property_readonly("rank", &HqReducer::rank)
      .def_property_readonly("world", &HqReducer::world)
      .def_property_readonly("comm_count", &HqReducer::comm_count);
}
