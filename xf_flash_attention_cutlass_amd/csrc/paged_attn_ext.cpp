// paged_attn_ext.cpp — the PyTorch op surface: pybind11 module `paged_attn`.
//
// Mirrors the reference's export.cpp (module export.cpp:1757-1764): `fwd` (mha_fwd,
// export.cpp:465-667), `varlen_fwd` (mha_varlen_fwd, :669-937), `fwd_kvcache`
// (mha_fwd_kvcache, :1433-1754) with the same argument lists and return tuples, plus `bwd`
// and `varlen_bwd`, which the reference has only as dead code (:939-1431).  `fwd_kvcache`
// also appends new K/V (with optional rotary) into the cache, which the reference validates
// but never executes (export.cpp:1585-1669, csrc/paged_attn.cpp:513-525).  Every op
// validates with TORCH_CHECK, allocates outputs, and calls the C ABI of
// libpaged-attention.so (include/paged_attn.h); errors reported by the C ABI are re-raised
// as RuntimeError.  Behaviour the reference gets wrong is fixed, not copied:
// LSE is always written; GQA decode is handled by the kernel's head packing instead of the
// transposed-view swap (:526-532); a [H]-shaped ALiBi vector is expanded rather than read
// out of bounds; dropout runs (Philox keep bits, rng_state = {seed, offset} as export.cpp
// returns it) instead of being silently ignored.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <ATen/hip/HIPGeneratorImpl.h>

#include <limits>

#include "paged_attn.h"

#define CHECK_DEVICE(x) TORCH_CHECK(x.is_cuda(), #x " must be on CUDA")
#define CHECK_SHAPE(x, ...) \
    TORCH_CHECK(x.sizes() == torch::IntArrayRef({__VA_ARGS__}), #x " must have shape (" #__VA_ARGS__ ")")
#define CHECK_CONTIGUOUS(x) TORCH_CHECK(x.is_contiguous(), #x " must be contiguous")

namespace {

void raise_if_failed(const char* op) {
    if (fmha_last_status() != 0) TORCH_CHECK(false, op, ": ", fmha_last_error());
}

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

int round8(int x) { return (x + 7) / 8 * 8; }

at::Tensor pad_last(const at::Tensor& t, int d_og) {
    if (d_og % 8 == 0) return t;
    return torch::nn::functional::pad(t, torch::nn::functional::PadFuncOptions({0, 8 - d_og % 8}));
}

// The kernels move 16-byte chunks (b128 buffer loads, LDS-DMA, 16-byte row stores): every base
// pointer must be 16-byte aligned and every row / head / batch stride a multiple of 16 bytes.
bool aligned16(const at::Tensor& t) {
    if ((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) != 0) return false;
    for (int i = 0; i + 1 < t.dim(); ++i)
        if (t.size(i) > 1 && (t.stride(i) * (int64_t)t.element_size()) % 16 != 0) return false;
    return true;
}

// contiguous AND 16-byte aligned (a view at an odd storage offset is copied)
at::Tensor dense(const at::Tensor& t) {
    at::Tensor c = t.contiguous();
    if (!aligned16(c)) c = c.clone(at::MemoryFormat::Contiguous);
    return c;
}

void check_qkv_dtype(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v) {
    auto dt = q.dtype();
    TORCH_CHECK(dt == torch::kFloat16 || dt == torch::kBFloat16,
                "FlashAttention only support fp16 and bf16 data type");
    TORCH_CHECK(k.dtype() == dt, "query and key must have the same dtype");
    TORCH_CHECK(v.dtype() == dt, "query and value must have the same dtype");
    CHECK_DEVICE(q); CHECK_DEVICE(k); CHECK_DEVICE(v);
    TORCH_CHECK(q.stride(-1) == 1, "Input tensor must have contiguous last dimension");
    TORCH_CHECK(k.stride(-1) == 1, "Input tensor must have contiguous last dimension");
    TORCH_CHECK(v.stride(-1) == 1, "Input tensor must have contiguous last dimension");
}

// ALiBi slopes as the C ABI wants them: fp32, [b, h] when batch > 1 (paged_attn.cpp:375).
at::Tensor alibi_for_c(c10::optional<at::Tensor>& a, int b, int h, int64_t* bstride) {
    if (!a.has_value()) { *bstride = 0; return at::Tensor(); }
    auto s = a.value();
    TORCH_CHECK(s.dtype() == torch::kFloat32, "ALiBi slopes must have dtype fp32");
    CHECK_DEVICE(s);
    TORCH_CHECK(s.stride(-1) == 1, "ALiBi slopes tensor must have contiguous last dimension");
    TORCH_CHECK(s.sizes() == torch::IntArrayRef({h}) || s.sizes() == torch::IntArrayRef({b, h}),
                "ALiBi slopes must have shape (num_heads) or (batch_size, num_heads)");
    if (s.dim() == 1) s = s.unsqueeze(0).expand({b, h});
    s = s.contiguous();
    *bstride = b > 1 ? h : 0;
    return s;
}

// Dropout: the key from torch's HIP generator (ATen/hip/HIPGeneratorImpl.h, whose generator
// class and Philox state keep their upstream names in this ROCm build: CUDAGeneratorImpl,
// PhiloxCudaState — no other spelling exists) as philox_cuda_state (export.cpp:616-627,
// flash_api_hip.cpp:509): outside stream capture the host seed / offset; under capture the
// generator's device seed / offset pointers, read by the kernels when the graph runs (so every
// replay draws a fresh mask).  rng_state is an int64 [2] on q's device, as upstream returns it;
// the forward kernel writes the key it used into it, and the backward reads it on the device.
at::Tensor dropout_rng(float p_dropout, c10::optional<at::Generator>& gen_, int64_t counter_offset,
                       const at::Device& dev) {
    auto rng = torch::empty({2}, torch::dtype(torch::kInt64).device(dev));
    if (p_dropout > 0.f) {
        auto gen = at::get_generator_or_default<at::CUDAGeneratorImpl>(gen_, at::cuda::detail::getDefaultCUDAGenerator());
        at::PhiloxCudaState st;
        {
            std::lock_guard<std::mutex> lock(gen->mutex_);
            st = gen->philox_cuda_state((uint64_t)counter_offset);
        }
        if (st.captured_) {
            fmha_set_rng_state(0, 0);
            fmha_set_rng_state_device(st.seed_.ptr, st.offset_.ptr, st.offset_intragraph_, rng.data_ptr<int64_t>());
        } else {
            fmha_set_rng_state(st.seed_.val, st.offset_.val);
            fmha_set_rng_state_device(nullptr, nullptr, 0, rng.data_ptr<int64_t>());
        }
    } else {
        fmha_set_rng_state(0, 0);
    }
    return rng;
}

// The backward's key: a device rng_state (the forward's) is read on the device (capturable);
// a host one (a caller's own {seed, offset}) is passed by value.
void dropout_rng_restore(float p_dropout, c10::optional<at::Tensor>& rng_state) {
    if (p_dropout <= 0.f) return;
    TORCH_CHECK(rng_state.has_value(), "backward with dropout needs the forward's rng_state");
    const at::Tensor& r0 = rng_state.value();
    TORCH_CHECK(r0.numel() == 2 && r0.scalar_type() == torch::kInt64, "rng_state must be int64 {seed, offset}");
    if (r0.is_cuda()) {
        TORCH_CHECK(r0.is_contiguous(), "rng_state must be contiguous");
        const int64_t* d = r0.data_ptr<int64_t>();
        fmha_set_rng_state(0, 0);
        fmha_set_rng_state_device(d, d + 1, 0, nullptr);
        return;
    }
    auto r = r0.contiguous();
    fmha_set_rng_state((uint64_t)r.data_ptr<int64_t>()[0], (uint64_t)r.data_ptr<int64_t>()[1]);
}

// Disarms the thread's device dropout key when the binding returns or throws: a check
// that fails after dropout_rng / dropout_rng_restore, or a forward with seqlen_k == 0 that runs no
// C entry, must not leave pointers to tensors about to be freed for a later direct C-ABI call.
struct RngDisarm {
    ~RngDisarm() { fmha_set_rng_state_device(nullptr, nullptr, 0, nullptr); }
};

at::Tensor sdmask_buffer(bool want, const at::TensorOptions& opts, int b, int h, int sq, int sk) {
    if (!want) return at::Tensor();
    auto r128 = [](int x) { return (x + 127) / 128 * 128; };
    return torch::empty({b, h, r128(sq), r128(sk)}, opts);
}

}  // namespace

std::vector<at::Tensor>
mha_fwd(at::Tensor& q, const at::Tensor& k, const at::Tensor& v, c10::optional<at::Tensor>& out_,
        c10::optional<at::Tensor>& alibi_slopes_, const float p_dropout, const float softmax_scale,
        bool is_causal, int window_size_left, int window_size_right, const float softcap,
        const bool return_softmax, c10::optional<at::Generator> gen_) {
    check_qkv_dtype(q, k, v);
    const auto sizes = q.sizes();
    TORCH_CHECK(q.dim() == 4, "q must be (batch, seqlen, heads, head_size)");
    const int batch_size = sizes[0];
    const int seqlen_q = sizes[1];
    const int num_heads = sizes[2];
    const int head_size_og = sizes[3];
    const int seqlen_k = k.size(1);
    const int num_heads_k = k.size(2);
    TORCH_CHECK(batch_size > 0, "batch size must be postive");
    TORCH_CHECK(head_size_og <= 256, "FlashAttention forward only supports head dimension at most 256");
    TORCH_CHECK(num_heads % num_heads_k == 0, "Number of heads in key/value must divide number of heads in query");
    TORCH_CHECK(p_dropout >= 0.f && p_dropout < 1.f, "p_dropout must be in [0, 1)");
    if (softcap > 0.f) { TORCH_CHECK(p_dropout == 0.f, "Softcapping does not support dropout for now"); }
    TORCH_CHECK(!return_softmax || p_dropout > 0.f, "return_softmax is only supported when p_dropout > 0.0");
    if (window_size_left >= seqlen_k) window_size_left = -1;
    if (window_size_right >= seqlen_k) window_size_right = -1;
    if (seqlen_q == 1 && !alibi_slopes_.has_value()) is_causal = false;
    if (is_causal) window_size_right = 0;
    CHECK_SHAPE(q, batch_size, seqlen_q, num_heads, head_size_og);
    CHECK_SHAPE(k, batch_size, seqlen_k, num_heads_k, head_size_og);
    CHECK_SHAPE(v, batch_size, seqlen_k, num_heads_k, head_size_og);

    // d % 8 == 0 and 16-byte aligned: strided views (head / batch slices, kvpacked kv[:, :, 0])
    // run in place through fmha_fwd_strided; otherwise the reference's padding to a multiple of
    // 8 (export.cpp:539-547) into aligned contiguous copies
    const bool strided = head_size_og % 8 == 0 && aligned16(q) && aligned16(k) && aligned16(v);
    at::Tensor q_padded = strided ? q : dense(pad_last(q, head_size_og));
    at::Tensor k_padded = strided ? k : dense(pad_last(k, head_size_og));
    at::Tensor v_padded = strided ? v : dense(pad_last(v, head_size_og));
    at::Tensor out;
    if (out_.has_value()) {
        out = out_.value();
        TORCH_CHECK(out.dtype() == q.dtype(), "Output must have the same dtype as inputs");
        CHECK_DEVICE(out);
        TORCH_CHECK(out.stride(-1) == 1, "Output tensor must have contiguous last dimension");
        CHECK_SHAPE(out, batch_size, seqlen_q, num_heads, head_size_og);
        if (head_size_og % 8 != 0 || !aligned16(out) || (!strided && !out.is_contiguous()))
            out = torch::empty_like(q_padded, at::MemoryFormat::Contiguous);
    } else {
        out = torch::empty_like(q_padded, at::MemoryFormat::Contiguous);
    }
    const int head_size = round8(head_size_og);
    const c10::DeviceGuard device_guard(q.device());
    auto opts = q.options();
    auto softmax_lse = torch::empty({batch_size, num_heads, seqlen_q}, opts.dtype(at::kFloat));
    at::Tensor p = sdmask_buffer(return_softmax, opts, batch_size, num_heads, seqlen_q, seqlen_k);
    auto rng_state = dropout_rng(p_dropout, gen_, (int64_t)batch_size * num_heads * 32, q.device());
    RngDisarm rng_disarm;
    int64_t alibi_bs = 0;
    at::Tensor alibi = alibi_for_c(alibi_slopes_, batch_size, num_heads, &alibi_bs);

    if (seqlen_k > 0 && strided) {
        const int64_t st[12] = {q.stride(0), q.stride(1), q.stride(2), k.stride(0), k.stride(1),
                                k.stride(2), v.stride(0), v.stride(1), v.stride(2), out.stride(0),
                                out.stride(1), out.stride(2)};
        fmha_fwd_strided(q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(),
                         alibi.defined() ? alibi.data_ptr() : nullptr, softmax_lse.data_ptr(),
                         seqlen_q, seqlen_k, batch_size, num_heads, num_heads_k, head_size, st,
                         softmax_scale, window_size_left, window_size_right, softcap,
                         q.dtype() == torch::kFloat16, 0, cur_stream(), p_dropout,
                         p.defined() ? p.data_ptr() : nullptr);
        raise_if_failed("fwd");
    } else if (seqlen_k > 0) {
        fmha_fwd(q_padded.data_ptr(), k_padded.data_ptr(), v_padded.data_ptr(), out.data_ptr(),
                 alibi.defined() ? alibi.data_ptr() : nullptr, seqlen_q, seqlen_k, batch_size,
                 num_heads, num_heads_k, head_size, p_dropout, cur_stream(), nullptr, softmax_scale,
                 p.defined() ? p.data_ptr() : nullptr, softmax_lse.data_ptr(), window_size_left,
                 window_size_right, softcap, return_softmax, q.dtype() == torch::kFloat16, 0);
        raise_if_failed("fwd");
    } else {
        out.zero_();
        softmax_lse.fill_(std::numeric_limits<float>::infinity());
    }
    at::Tensor out_padded = out;
    if (head_size_og % 8 != 0) out = out.index({"...", torch::indexing::Slice(torch::indexing::None, head_size_og)});
    if (out_.has_value() && !out_.value().is_same(out)) out_.value().copy_(out), out = out_.value();
    return {out, q_padded, k_padded, v_padded, out_padded, softmax_lse, p, rng_state};
}

std::vector<at::Tensor>
mha_varlen_fwd(at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
               c10::optional<at::Tensor>& out_, const at::Tensor& cu_seqlens_q,
               const at::Tensor& cu_seqlens_k, c10::optional<at::Tensor>& seqused_k,
               c10::optional<at::Tensor>& block_table_, c10::optional<at::Tensor>& alibi_slopes_,
               int max_seqlen_q, const int max_seqlen_k, const float p_dropout,
               const float softmax_scale, const bool zero_tensors, bool is_causal,
               int window_size_left, int window_size_right, const float softcap,
               const bool return_softmax, c10::optional<at::Generator> gen_) {
    check_qkv_dtype(q, k, v);
    TORCH_CHECK(cu_seqlens_q.dtype() == torch::kInt32, "cu_seqlens_q must have dtype int32");
    TORCH_CHECK(cu_seqlens_k.dtype() == torch::kInt32, "cu_seqlens_k must have dtype int32");
    CHECK_DEVICE(cu_seqlens_q); CHECK_DEVICE(cu_seqlens_k);
    CHECK_CONTIGUOUS(cu_seqlens_q); CHECK_CONTIGUOUS(cu_seqlens_k);
    at::Tensor block_table;
    const bool paged_KV = block_table_.has_value();
    if (paged_KV) {
        block_table = block_table_.value();
        CHECK_DEVICE(block_table);
        TORCH_CHECK(block_table.dtype() == torch::kInt32, "block_table must have dtype torch.int32");
        TORCH_CHECK(block_table.stride(-1) == 1, "block_table must have contiguous last dimension");
    }
    const auto sizes = q.sizes();
    const int batch_size = cu_seqlens_q.numel() - 1;
    const int num_heads = sizes[1];
    const int head_size_og = sizes[2];
    const int num_heads_k = paged_KV ? k.size(2) : k.size(1);
    const int total_q = sizes[0];
    TORCH_CHECK(batch_size > 0, "batch size must be positive");
    TORCH_CHECK(head_size_og <= 256, "FlashAttention forward only supports head dimension at most 256");
    TORCH_CHECK(num_heads % num_heads_k == 0, "Number of heads in key/value must divide number of heads in query");
    TORCH_CHECK(p_dropout >= 0.f && p_dropout < 1.f, "p_dropout must be in [0, 1)");
    if (softcap > 0.f) { TORCH_CHECK(p_dropout == 0.f, "Softcapping does not support dropout for now"); }
    TORCH_CHECK(!return_softmax || p_dropout > 0.f, "return_softmax is only supported when p_dropout > 0.0");
    TORCH_CHECK(p_dropout == 0.f || !paged_KV, "dropout over a paged K/V cache is not supported");
    const int max_num_blocks_per_seq = !paged_KV ? 0 : block_table.size(1);
    const int num_blocks = !paged_KV ? 0 : k.size(0);
    const int page_block_size = !paged_KV ? 1 : k.size(1);
    if (max_seqlen_q == 1 && !alibi_slopes_.has_value()) is_causal = false;
    if (is_causal) window_size_right = 0;
    if (window_size_left >= max_seqlen_k) window_size_left = -1;
    if (window_size_right >= max_seqlen_k) window_size_right = -1;
    CHECK_SHAPE(q, total_q, num_heads, head_size_og);
    if (!paged_KV) {
        const int total_k = k.size(0);
        CHECK_SHAPE(k, total_k, num_heads_k, head_size_og);
        CHECK_SHAPE(v, total_k, num_heads_k, head_size_og);
    } else {
        CHECK_SHAPE(k, num_blocks, page_block_size, num_heads_k, head_size_og);
        CHECK_SHAPE(v, num_blocks, page_block_size, num_heads_k, head_size_og);
        CHECK_SHAPE(block_table, batch_size, max_num_blocks_per_seq);
    }
    CHECK_SHAPE(cu_seqlens_q, batch_size + 1);
    CHECK_SHAPE(cu_seqlens_k, batch_size + 1);
    at::Tensor seqused;
    if (seqused_k.has_value()) {
        seqused = seqused_k.value();
        TORCH_CHECK(seqused.dtype() == torch::kInt32, "seqused_k must have dtype int32");
        TORCH_CHECK(seqused.is_cuda(), "seqused_k must be on CUDA device");
        TORCH_CHECK(seqused.is_contiguous(), "seqused_k must be contiguous");
        CHECK_SHAPE(seqused, batch_size);
    }
    at::Tensor q_padded = dense(pad_last(q, head_size_og));
    at::Tensor k_padded = dense(pad_last(k, head_size_og));
    at::Tensor v_padded = dense(pad_last(v, head_size_og));
    at::Tensor out;
    if (out_.has_value()) {
        out = out_.value();
        TORCH_CHECK(out.dtype() == q.dtype(), "Output must have the same dtype as inputs");
        CHECK_DEVICE(out);
        TORCH_CHECK(out.stride(-1) == 1, "Output tensor must have contiguous last dimension");
        CHECK_SHAPE(out, sizes[0], sizes[1], head_size_og);
        if (head_size_og % 8 != 0 || !out.is_contiguous() || !aligned16(out)) out = torch::empty_like(q_padded);
    } else {
        out = torch::empty_like(q_padded);
    }
    const int head_size = round8(head_size_og);
    const c10::DeviceGuard device_guard(q.device());
    auto opts = q.options();
    auto softmax_lse = torch::empty({num_heads, total_q}, opts.dtype(at::kFloat));
    at::Tensor p = sdmask_buffer(return_softmax, opts, batch_size, num_heads, max_seqlen_q, max_seqlen_k);
    auto rng_state = dropout_rng(p_dropout, gen_, (int64_t)batch_size * num_heads * 32, q.device());
    RngDisarm rng_disarm;
    if (zero_tensors) {
        out.zero_();
        softmax_lse.fill_(-std::numeric_limits<float>::infinity());
    }
    int64_t alibi_bs = 0;
    at::Tensor alibi = alibi_for_c(alibi_slopes_, batch_size, num_heads, &alibi_bs);
    if (max_seqlen_k > 0) {
        fmha_varlen_fwd_ex(q_padded.data_ptr(), k_padded.data_ptr(), v_padded.data_ptr(),
                           out.data_ptr(), softmax_lse.data_ptr(), cu_seqlens_q.data_ptr(),
                           cu_seqlens_k.data_ptr(), seqused.defined() ? seqused.data_ptr() : nullptr,
                           paged_KV ? block_table.data_ptr() : nullptr,
                           paged_KV ? (int)block_table.stride(0) : 0, page_block_size,
                           alibi.defined() ? alibi.data_ptr() : nullptr, (int)alibi_bs,
                           max_seqlen_q, max_seqlen_k, total_q, batch_size, num_heads, num_heads_k,
                           head_size, softmax_scale, window_size_left, window_size_right, softcap,
                           q.dtype() == torch::kFloat16, cur_stream(), p_dropout,
                           p.defined() ? p.data_ptr() : nullptr);
        raise_if_failed("varlen_fwd");
    } else {
        out.zero_();
        softmax_lse.fill_(std::numeric_limits<float>::infinity());
    }
    at::Tensor out_padded = out;
    if (head_size_og % 8 != 0) out = out.index({"...", torch::indexing::Slice(torch::indexing::None, head_size_og)});
    if (out_.has_value() && !out_.value().is_same(out)) out_.value().copy_(out), out = out_.value();
    return {out, q_padded, k_padded, v_padded, out_padded, softmax_lse, p, rng_state};
}

std::vector<at::Tensor>
mha_fwd_kvcache(at::Tensor& q, const at::Tensor& kcache, const at::Tensor& vcache,
                c10::optional<const at::Tensor>& k_, c10::optional<const at::Tensor>& v_,
                c10::optional<const at::Tensor>& seqlens_k_,
                c10::optional<const at::Tensor>& rotary_cos_,
                c10::optional<const at::Tensor>& rotary_sin_,
                c10::optional<const at::Tensor>& cache_batch_idx_,
                c10::optional<at::Tensor>& block_table_, c10::optional<at::Tensor>& alibi_slopes_,
                c10::optional<at::Tensor>& out_, const float softmax_scale, bool is_causal,
                int window_size_left, int window_size_right, const float softcap,
                bool is_rotary_interleaved, int num_splits,
                c10::optional<const at::Tensor>& cache_leftpad_) {
    check_qkv_dtype(q, kcache, vcache);
    const bool append = k_.has_value();
    const bool local_or_causal = is_causal || window_size_left >= 0 || window_size_right >= 0;
    at::Tensor block_table;
    const bool paged_KV = block_table_.has_value();
    if (paged_KV) {
        block_table = block_table_.value();
        CHECK_DEVICE(block_table);
        TORCH_CHECK(block_table.dtype() == torch::kInt32, "block_table must have dtype torch.int32");
        TORCH_CHECK(block_table.stride(-1) == 1, "block_table must have contiguous last dimension");
    }
    const auto sizes = q.sizes();
    const int batch_size = sizes[0];
    const int seqlen_q = sizes[1];
    const int num_heads = sizes[2];
    const int head_size_og = sizes[3];
    const int max_num_blocks_per_seq = !paged_KV ? 1 : block_table.size(1);
    const int num_blocks = !paged_KV ? kcache.size(0) : kcache.size(0);
    const int page_block_size = !paged_KV ? kcache.size(1) : kcache.size(1);
    const int seqlen_k = max_num_blocks_per_seq * page_block_size;
    const int num_heads_k = kcache.size(2);
    TORCH_CHECK(batch_size > 0, "batch size must be positive");
    TORCH_CHECK(head_size_og <= 256, "FlashAttention forward only supports head dimension at most 256");
    TORCH_CHECK(num_heads % num_heads_k == 0, "Number of heads in key/value must divide number of heads in query");
    if (seqlen_q == 1 && !alibi_slopes_.has_value()) is_causal = false;
    if (is_causal) window_size_right = 0;
    if (window_size_left >= seqlen_k) window_size_left = -1;
    if (window_size_right >= seqlen_k) window_size_right = -1;
    CHECK_SHAPE(q, batch_size, seqlen_q, num_heads, head_size_og);
    if (!paged_KV) {
        // Dense cache [batch_cache, seqlen_k, hk, d]: one "page" per sequence (the reference's
        // non-paged branch dereferences an undefined block_table, export.cpp:1711); the page of
        // batch b is cache_batch_idx[b] when given, else b.
        const int bc = kcache.size(0);
        CHECK_SHAPE(kcache, bc, page_block_size, num_heads_k, head_size_og);
        CHECK_SHAPE(vcache, bc, page_block_size, num_heads_k, head_size_og);
        if (cache_batch_idx_.has_value()) {
            auto idx = cache_batch_idx_.value();
            CHECK_DEVICE(idx); CHECK_CONTIGUOUS(idx);
            TORCH_CHECK(idx.scalar_type() == torch::kInt32, "cache_batch_idx must have dtype int32");
            CHECK_SHAPE(idx, batch_size);
            block_table = idx.view({batch_size, 1});
        } else {
            TORCH_CHECK(bc == batch_size, "k_cache batch must equal q batch without cache_batch_idx");
            block_table = torch::arange(batch_size, q.options().dtype(torch::kInt32)).view({batch_size, 1});
        }
    } else {
        TORCH_CHECK(!cache_batch_idx_.has_value(),
                    "cache_batch_idx cannot be combined with a paged KV cache");
        CHECK_SHAPE(kcache, num_blocks, page_block_size, num_heads_k, head_size_og);
        CHECK_SHAPE(vcache, num_blocks, page_block_size, num_heads_k, head_size_og);
        CHECK_SHAPE(block_table, batch_size, max_num_blocks_per_seq);
    }
    at::Tensor q_padded = dense(pad_last(q, head_size_og));
    at::Tensor kc = dense(pad_last(kcache, head_size_og));
    at::Tensor vc = dense(pad_last(vcache, head_size_og));
    at::Tensor out;
    if (out_.has_value()) {
        out = out_.value();
        TORCH_CHECK(out.dtype() == q.dtype(), "Output must have the same dtype as inputs");
        CHECK_DEVICE(out);
        TORCH_CHECK(out.stride(-1) == 1, "Output tensor must have contiguous last dimension");
        CHECK_SHAPE(out, batch_size, seqlen_q, num_heads, head_size_og);
        if (head_size_og % 8 != 0 || !out.is_contiguous() || !aligned16(out)) out = torch::empty_like(q_padded);
    } else {
        out = torch::empty_like(q_padded);
    }
    const int head_size = round8(head_size_og);
    const c10::DeviceGuard device_guard(q.device());
    auto opts = q.options();
    auto softmax_lse = torch::empty({batch_size, num_heads, seqlen_q}, opts.dtype(at::kFloat));
    at::Tensor seqlens;
    if (seqlens_k_.has_value()) {
        seqlens = seqlens_k_.value();
        TORCH_CHECK(seqlens.dtype() == torch::kInt32, "seqlens_k must have dtype int32");
        CHECK_DEVICE(seqlens);
        CHECK_CONTIGUOUS(seqlens);
        CHECK_SHAPE(seqlens, batch_size);
    }
    // cache_leftpad (flash-attn's leftpad_k, commented out at export.cpp:1443,1627-1634): batch b's
    // sequence is cache rows [leftpad[b], seqlens_k[b]); non-paged caches only, as there
    at::Tensor leftpad;
    if (cache_leftpad_.has_value()) {
        leftpad = cache_leftpad_.value();
        TORCH_CHECK(!paged_KV, "We don't support Paged KV and leftpad_k running at the same time yet");
        TORCH_CHECK(leftpad.dtype() == torch::kInt32, "leftpad_k must have dtype int32");
        CHECK_DEVICE(leftpad);
        CHECK_CONTIGUOUS(leftpad);
        CHECK_SHAPE(leftpad, batch_size);
        TORCH_CHECK(seqlens.defined(), "cache_leftpad needs seqlens_k");
    }
    int64_t alibi_bs = 0;
    at::Tensor alibi = alibi_for_c(alibi_slopes_, batch_size, num_heads, &alibi_bs);
    at::Tensor q_attn = q_padded;
    if (append) {
        // write the new rows into the cache in place (+ rotary on k and q), then attend over the
        // cache with the grown lengths (export.cpp:1585-1669 validation)
        TORCH_CHECK(v_.has_value(), "If key is supplied, value must also be passed in");
        TORCH_CHECK(seqlens.defined(), "If key is supplied, seqlens_k must also be passed in");
        const at::Tensor& kn = k_.value();
        const at::Tensor& vn = v_.value();
        TORCH_CHECK(kn.dtype() == q.dtype(), "Key must have the same dtype as query");
        TORCH_CHECK(vn.dtype() == q.dtype(), "Value must have the same dtype as query");
        CHECK_DEVICE(kn); CHECK_DEVICE(vn); CHECK_CONTIGUOUS(kn); CHECK_CONTIGUOUS(vn);
        const int seqlen_new = kn.size(1);
        CHECK_SHAPE(kn, batch_size, seqlen_new, num_heads_k, head_size_og);
        CHECK_SHAPE(vn, batch_size, seqlen_new, num_heads_k, head_size_og);
        TORCH_CHECK(seqlen_q <= seqlen_k, "If key is supplied, it must have seqlen <= the seqlen of the KV cache");
        TORCH_CHECK(head_size_og % 8 == 0 && kcache.is_contiguous() && vcache.is_contiguous(),
                    "appending needs contiguous caches with head_size a multiple of 8 (updated in place)");
        int rotary_dim = 0;
        at::Tensor cos, sin, q_rot;
        if (rotary_cos_.has_value()) {
            TORCH_CHECK(rotary_sin_.has_value(), "If rotary cos is provided, rotary sin must also be provided");
            cos = rotary_cos_.value();
            sin = rotary_sin_.value();
            CHECK_DEVICE(cos); CHECK_DEVICE(sin); CHECK_CONTIGUOUS(cos); CHECK_CONTIGUOUS(sin);
            rotary_dim = cos.size(1) * 2;
            TORCH_CHECK(rotary_dim <= head_size_og, "rotary_dim must be <= headdim");
            TORCH_CHECK(rotary_dim % 16 == 0, "Only rotary dimensions divisible by 16 are currently supported");
            TORCH_CHECK(cos.size(0) >= seqlen_k, "cos/sin seqlen must be at least the seqlen of KV cache");
            CHECK_SHAPE(sin, cos.size(0), rotary_dim / 2);
            TORCH_CHECK(cos.scalar_type() == q.scalar_type() && sin.scalar_type() == q.scalar_type(),
                        "rotary_cos/sin must have the same dtype as query");
            q_rot = torch::empty_like(q_padded);
        }
        auto seqlens_new = torch::empty_like(seqlens);
        fmha_kvcache_append(q_padded.data_ptr(), q_rot.defined() ? q_rot.data_ptr() : nullptr,
                            kc.data_ptr(), vc.data_ptr(), kn.data_ptr(), vn.data_ptr(), seqlen_new,
                            block_table.data_ptr(), (int)block_table.stride(0), page_block_size,
                            seqlens.data_ptr(), seqlens_new.data_ptr(),
                            cos.defined() ? cos.data_ptr() : nullptr,
                            sin.defined() ? sin.data_ptr() : nullptr, rotary_dim,
                            is_rotary_interleaved, local_or_causal, batch_size, seqlen_q,
                            num_heads, num_heads_k, head_size, q.dtype() == torch::kFloat16,
                            cur_stream());
        raise_if_failed("fwd_kvcache (append)");
        seqlens = seqlens_new;
        if (q_rot.defined()) q_attn = q_rot;
    } else {
        TORCH_CHECK(!rotary_cos_.has_value(),
                    "If rotary cos/sin are provided, new key / value to be appended to KV cache must also be provided");
    }
    fmha_page_kvcache_fwd_ex(q_attn.data_ptr(), kc.data_ptr(), vc.data_ptr(), out.data_ptr(),
                             softmax_lse.data_ptr(), block_table.data_ptr(),
                             (int)block_table.stride(0),
                             seqlens.defined() ? seqlens.data_ptr() : nullptr, seqlen_q, seqlen_k,
                             batch_size, num_heads, num_heads_k, head_size, page_block_size,
                             softmax_scale, window_size_left, window_size_right, softcap,
                             alibi.defined() ? alibi.data_ptr() : nullptr, (int)alibi_bs,
                             num_splits, 0, 1.f, 1.f,
                             leftpad.defined() ? leftpad.data_ptr() : nullptr,
                             q.dtype() == torch::kFloat16, cur_stream());
    raise_if_failed("fwd_kvcache");
    if (head_size_og % 8 != 0) out = out.index({"...", torch::indexing::Slice(torch::indexing::None, head_size_og)});
    if (out_.has_value() && !out_.value().is_same(out)) out_.value().copy_(out), out = out_.value();
    return {out, softmax_lse};
}

// Gradient outputs (export.cpp:1037-1060): a caller-given tensor must match q/k/v in dtype,
// device and shape; a non-contiguous one is computed into a contiguous temporary and copied
// back by grad_writeback.
static at::Tensor grad_out(c10::optional<at::Tensor>& t, const at::Tensor& like) {
    if (t.has_value()) {
        const at::Tensor& x = t.value();
        TORCH_CHECK(x.dtype() == like.dtype(), "gradient must have the same dtype as its input");
        CHECK_DEVICE(x);
        TORCH_CHECK(x.sizes() == like.sizes(), "gradient has the wrong shape");
        if (x.is_contiguous() && aligned16(x)) return x;
    }
    return torch::empty_like(like, like.options().memory_format(at::MemoryFormat::Contiguous));
}
static void grad_writeback(c10::optional<at::Tensor>& t, at::Tensor& g) {
    if (t.has_value() && !t.value().is_same(g)) { t.value().copy_(g); g = t.value(); }
}

std::vector<at::Tensor>
mha_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
        const at::Tensor& out, const at::Tensor& softmax_lse, c10::optional<at::Tensor>& dq_,
        c10::optional<at::Tensor>& dk_, c10::optional<at::Tensor>& dv_,
        c10::optional<at::Tensor>& alibi_slopes_, const float p_dropout,
        const float softmax_scale, const bool is_causal, int window_size_left,
        int window_size_right, const float softcap, const bool deterministic,
        c10::optional<at::Generator> /*gen_*/, c10::optional<at::Tensor>& rng_state) {
    check_qkv_dtype(q, k, v);
    if (is_causal) window_size_right = 0;
    TORCH_CHECK(out.dtype() == q.dtype(), "query and out must have the same dtype");
    TORCH_CHECK(dout.dtype() == q.dtype(), "query and dout must have the same dtype");
    CHECK_DEVICE(out); CHECK_DEVICE(dout); CHECK_DEVICE(softmax_lse);
    TORCH_CHECK(p_dropout >= 0.f && p_dropout < 1.f, "p_dropout must be in [0, 1)");
    if (softcap > 0.f) { TORCH_CHECK(p_dropout == 0.f, "Softcapping does not support dropout for now"); }
    dropout_rng_restore(p_dropout, rng_state);
    RngDisarm rng_disarm;
    const auto sizes = q.sizes();
    const int batch_size = sizes[0];
    const int seqlen_q = sizes[1];
    const int num_heads = sizes[2];
    const int head_size_og = dout.size(3);
    const int head_size = sizes[3];
    const int seqlen_k = k.size(1);
    const int num_heads_k = k.size(2);
    TORCH_CHECK(batch_size > 0, "batch size must be positive");
    TORCH_CHECK(head_size % 8 == 0, "head_size should be a multiple of 8");
    TORCH_CHECK(head_size <= 256, "FlashAttention backward only supports head dimension at most 256");
    TORCH_CHECK(num_heads % num_heads_k == 0, "Number of heads in key/value must divide number of heads in query");
    TORCH_CHECK(head_size == round8(head_size_og), "head_size must be head_size_og rounded to a multiple of 8");
    if (window_size_left >= seqlen_k) window_size_left = -1;
    if (window_size_right >= seqlen_k) window_size_right = -1;
    CHECK_SHAPE(q, batch_size, seqlen_q, num_heads, head_size);
    CHECK_SHAPE(k, batch_size, seqlen_k, num_heads_k, head_size);
    CHECK_SHAPE(v, batch_size, seqlen_k, num_heads_k, head_size);
    CHECK_SHAPE(out, batch_size, seqlen_q, num_heads, head_size);
    CHECK_SHAPE(dout, batch_size, seqlen_q, num_heads, head_size_og);
    CHECK_SHAPE(softmax_lse, batch_size, num_heads, seqlen_q);
    at::Tensor dq = grad_out(dq_, q), dk = grad_out(dk_, k), dv = grad_out(dv_, v);
    at::Tensor dout_padded = dense(pad_last(dout, head_size_og));
    const c10::DeviceGuard device_guard(q.device());
    auto opts = q.options();
    auto softmax_d = torch::empty({batch_size, num_heads, seqlen_q}, opts.dtype(at::kFloat));
    int64_t alibi_bs = 0;
    at::Tensor alibi = alibi_for_c(alibi_slopes_, batch_size, num_heads, &alibi_bs);
    auto qc = dense(q), kc = dense(k), vc = dense(v), oc = dense(out);
    auto lse = softmax_lse.contiguous();
    const size_t ws = fmha_bwd_workspace_size(seqlen_q, seqlen_k, batch_size, num_heads, num_heads_k,
                                              head_size, deterministic);
    at::Tensor workspace = torch::empty({(int64_t)ws}, opts.dtype(torch::kUInt8));
    if (seqlen_q > 0) {
        fmha_bwd(dout_padded.data_ptr(), qc.data_ptr(), kc.data_ptr(), vc.data_ptr(), oc.data_ptr(),
                 lse.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(),
                 alibi.defined() ? alibi.data_ptr() : nullptr, softmax_d.data_ptr(), seqlen_q,
                 seqlen_k, batch_size, num_heads, num_heads_k, head_size, p_dropout, softmax_scale,
                 window_size_left, window_size_right, softcap, deterministic,
                 q.dtype() == torch::kFloat16, cur_stream(), workspace.data_ptr(), ws);
        raise_if_failed("bwd");
    } else {
        dk.zero_(); dv.zero_(); softmax_d.zero_();
    }
    grad_writeback(dq_, dq); grad_writeback(dk_, dk); grad_writeback(dv_, dv);
    if (head_size_og % 8 != 0) {
        using torch::indexing::Slice; using torch::indexing::None;
        dq = dq.index({"...", Slice(None, head_size_og)});
        dk = dk.index({"...", Slice(None, head_size_og)});
        dv = dv.index({"...", Slice(None, head_size_og)});
    }
    return {dq, dk, dv, softmax_d};
}

std::vector<at::Tensor>
mha_varlen_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k,
               const at::Tensor& v, const at::Tensor& out, const at::Tensor& softmax_lse,
               c10::optional<at::Tensor>& dq_, c10::optional<at::Tensor>& dk_,
               c10::optional<at::Tensor>& dv_, const at::Tensor& cu_seqlens_q,
               const at::Tensor& cu_seqlens_k, c10::optional<at::Tensor>& alibi_slopes_,
               const int max_seqlen_q, const int max_seqlen_k, const float p_dropout,
               const float softmax_scale, const bool zero_tensors, const bool is_causal,
               int window_size_left, int window_size_right, const float softcap,
               const bool deterministic, c10::optional<at::Generator> /*gen_*/,
               c10::optional<at::Tensor>& rng_state) {
    check_qkv_dtype(q, k, v);
    if (is_causal) window_size_right = 0;
    TORCH_CHECK(p_dropout >= 0.f && p_dropout < 1.f, "p_dropout must be in [0, 1)");
    if (softcap > 0.f) { TORCH_CHECK(p_dropout == 0.f, "Softcapping does not support dropout for now"); }
    dropout_rng_restore(p_dropout, rng_state);
    RngDisarm rng_disarm;
    TORCH_CHECK(cu_seqlens_q.dtype() == torch::kInt32, "cu_seqlens_q must have dtype int32");
    TORCH_CHECK(cu_seqlens_k.dtype() == torch::kInt32, "cu_seqlens_k must have dtype int32");
    const int batch_size = cu_seqlens_q.numel() - 1;
    const int total_q = q.size(0), num_heads = q.size(1), head_size = q.size(2);
    const int total_k = k.size(0), num_heads_k = k.size(1);
    const int head_size_og = dout.size(2);
    TORCH_CHECK(head_size % 8 == 0, "head_size should be a multiple of 8");
    TORCH_CHECK(head_size <= 256, "FlashAttention backward only supports head dimension at most 256");
    TORCH_CHECK(num_heads % num_heads_k == 0, "Number of heads in key/value must divide number of heads in query");
    if (window_size_left >= max_seqlen_k) window_size_left = -1;
    if (window_size_right >= max_seqlen_k) window_size_right = -1;
    CHECK_SHAPE(softmax_lse, num_heads, total_q);
    CHECK_SHAPE(k, total_k, num_heads_k, head_size);
    CHECK_SHAPE(v, total_k, num_heads_k, head_size);
    CHECK_SHAPE(out, total_q, num_heads, head_size);
    CHECK_SHAPE(dout, total_q, num_heads, head_size_og);
    at::Tensor dq = grad_out(dq_, q), dk = grad_out(dk_, k), dv = grad_out(dv_, v);
    at::Tensor dout_padded = dense(pad_last(dout, head_size_og));
    const c10::DeviceGuard device_guard(q.device());
    auto opts = q.options();
    auto softmax_d = torch::empty({num_heads, total_q}, opts.dtype(at::kFloat));
    int64_t alibi_bs = 0;
    at::Tensor alibi = alibi_for_c(alibi_slopes_, batch_size, num_heads, &alibi_bs);
    auto qc = dense(q), kc = dense(k), vc = dense(v), oc = dense(out);
    auto lse = softmax_lse.contiguous();
    const size_t ws = fmha_varlen_bwd_workspace_size(total_q, max_seqlen_k, batch_size, num_heads,
                                                     num_heads_k, head_size, deterministic);
    at::Tensor workspace = torch::empty({(int64_t)ws}, opts.dtype(torch::kUInt8));
    fmha_varlen_bwd(dout_padded.data_ptr(), qc.data_ptr(), kc.data_ptr(), vc.data_ptr(),
                    oc.data_ptr(), lse.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(),
                    cu_seqlens_q.data_ptr(), cu_seqlens_k.data_ptr(),
                    alibi.defined() ? alibi.data_ptr() : nullptr, (int)alibi_bs, max_seqlen_q,
                    max_seqlen_k, total_q, total_k, batch_size, num_heads, num_heads_k, head_size,
                    softmax_scale, window_size_left, window_size_right, softcap, deterministic,
                    q.dtype() == torch::kFloat16, cur_stream(), workspace.data_ptr(), ws,
                    softmax_d.data_ptr(), p_dropout);
    raise_if_failed("varlen_bwd");
    (void)zero_tensors;
    grad_writeback(dq_, dq); grad_writeback(dk_, dk); grad_writeback(dv_, dv);
    if (head_size_og % 8 != 0) {
        using torch::indexing::Slice; using torch::indexing::None;
        dq = dq.index({"...", Slice(None, head_size_og)});
        dk = dk.index({"...", Slice(None, head_size_og)});
        dv = dv.index({"...", Slice(None, head_size_og)});
    }
    return {dq, dk, dv, softmax_d};
}

// Paged decode over an fp8 (OCP e4m3fn) K/V cache with per-tensor dequant scales — an
// extension the reference lacks.  kcache/vcache: float8_e4m3fn (or uint8 bytes)
// [num_blocks, page, hk, d]; returns {out, softmax_lse}.
std::vector<at::Tensor>
mha_fwd_kvcache_fp8(at::Tensor& q, const at::Tensor& kcache, const at::Tensor& vcache,
                    const at::Tensor& seqlens_k, const at::Tensor& block_table, const float k_scale,
                    const float v_scale, const float softmax_scale, bool is_causal,
                    int window_size_left, int window_size_right, int num_splits) {
    auto dt = q.dtype();
    TORCH_CHECK(dt == torch::kFloat16 || dt == torch::kBFloat16, "q must be fp16 or bf16");
    TORCH_CHECK(kcache.element_size() == 1 && vcache.element_size() == 1, "fp8 K/V cache expected");
    CHECK_DEVICE(q); CHECK_DEVICE(kcache); CHECK_DEVICE(vcache); CHECK_DEVICE(block_table); CHECK_DEVICE(seqlens_k);
    CHECK_CONTIGUOUS(kcache); CHECK_CONTIGUOUS(vcache);
    TORCH_CHECK(block_table.dtype() == torch::kInt32 && seqlens_k.dtype() == torch::kInt32,
                "block_table / seqlens_k must be int32");
    const int batch_size = q.size(0), seqlen_q = q.size(1), num_heads = q.size(2), d = q.size(3);
    const int page = kcache.size(1), num_heads_k = kcache.size(2);
    TORCH_CHECK(kcache.size(3) == d && d % 8 == 0 && d <= 256, "head_size must be a multiple of 8 and <= 256");
    TORCH_CHECK(num_heads % num_heads_k == 0, "Number of heads in key/value must divide number of heads in query");
    CHECK_SHAPE(block_table, batch_size, block_table.size(1));
    CHECK_SHAPE(seqlens_k, batch_size);
    const int seqlen_k = block_table.size(1) * page;
    if (seqlen_q == 1) is_causal = false;
    if (is_causal) window_size_right = 0;
    if (window_size_left >= seqlen_k) window_size_left = -1;
    if (window_size_right >= seqlen_k) window_size_right = -1;
    const c10::DeviceGuard device_guard(q.device());
    auto qc = dense(q);
    auto out = torch::empty_like(qc);
    auto lse = torch::empty({batch_size, num_heads, seqlen_q}, q.options().dtype(at::kFloat));
    auto bt = block_table.contiguous();
    fmha_page_kvcache_fwd_ex(qc.data_ptr(), kcache.data_ptr(), vcache.data_ptr(), out.data_ptr(),
                             lse.data_ptr(), bt.data_ptr(), (int)bt.stride(0), seqlens_k.data_ptr(),
                             seqlen_q, seqlen_k, batch_size, num_heads, num_heads_k, d, page,
                             softmax_scale, window_size_left, window_size_right, 0.f, nullptr, 0,
                             num_splits, 1, k_scale, v_scale, nullptr, dt == torch::kFloat16,
                             cur_stream());
    raise_if_failed("fwd_kvcache_fp8");
    return {out, lse};
}

// fp8 e4m3fn Q/K/V forward (extension): q [b, sq, h, 128], k/v [b, sk, hk, 128] as
// float8_e4m3fn (or uint8 bytes) with per-tensor descales; returns {out (out_dtype), lse}.
std::vector<at::Tensor>
mha_fwd_fp8(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
            c10::optional<at::Tensor>& out_, const float q_scale, const float k_scale,
            const float v_scale, const float softmax_scale, bool is_causal, int window_size_left,
            int window_size_right, const bool out_fp16) {
    TORCH_CHECK(q.element_size() == 1 && k.element_size() == 1 && v.element_size() == 1,
                "fp8 forward: q, k and v must be float8_e4m3fn (or uint8 bytes)");
    CHECK_DEVICE(q); CHECK_DEVICE(k); CHECK_DEVICE(v);
    CHECK_CONTIGUOUS(q); CHECK_CONTIGUOUS(k); CHECK_CONTIGUOUS(v);
    TORCH_CHECK(q.dim() == 4 && k.dim() == 4 && v.dim() == 4, "q, k, v must be [b, s, h, d]");
    const int batch_size = q.size(0), seqlen_q = q.size(1), num_heads = q.size(2), d = q.size(3);
    const int seqlen_k = k.size(1), num_heads_k = k.size(2);
    TORCH_CHECK(d == 128, "fp8 forward supports head_size 128");
    CHECK_SHAPE(k, batch_size, seqlen_k, num_heads_k, d);
    CHECK_SHAPE(v, batch_size, seqlen_k, num_heads_k, d);
    TORCH_CHECK(num_heads % num_heads_k == 0, "Number of heads in key/value must divide number of heads in query");
    if (seqlen_q == 1) is_causal = false;
    if (is_causal) window_size_right = 0;
    if (window_size_left >= seqlen_k) window_size_left = -1;
    if (window_size_right >= seqlen_k) window_size_right = -1;
    const c10::DeviceGuard device_guard(q.device());
    const auto odt = out_fp16 ? torch::kFloat16 : torch::kBFloat16;
    at::Tensor out;
    if (out_.has_value()) {
        out = out_.value();
        TORCH_CHECK(out.dtype() == odt, "out has the wrong dtype");
        CHECK_DEVICE(out); CHECK_CONTIGUOUS(out);
        CHECK_SHAPE(out, batch_size, seqlen_q, num_heads, d);
    } else {
        out = torch::empty({batch_size, seqlen_q, num_heads, d}, q.options().dtype(odt));
    }
    auto lse = torch::empty({batch_size, num_heads, seqlen_q}, q.options().dtype(at::kFloat));
    fmha_fwd_fp8(q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), lse.data_ptr(), q_scale,
                 k_scale, v_scale, seqlen_q, seqlen_k, batch_size, num_heads, num_heads_k, d,
                 softmax_scale, window_size_left, window_size_right, out_fp16, cur_stream());
    raise_if_failed("fwd_fp8");
    return {out, lse};
}

PYBIND11_MODULE(paged_attn, m) {
    m.doc() = "FlashAttention for MI355X (gfx950): hand-written HIP kernels behind the paged_attn C ABI";
    m.def("fwd", &mha_fwd, "Forward pass");
    m.def("varlen_fwd", &mha_varlen_fwd, "Forward pass (variable length)");
    // the reference's positional signature (export.cpp:1757) plus an optional trailing
    // cache_leftpad
    m.def("fwd_kvcache", &mha_fwd_kvcache, "Forward pass, with KV-cache", py::arg("q"),
          py::arg("kcache"), py::arg("vcache"), py::arg("k"), py::arg("v"), py::arg("seqlens_k"),
          py::arg("rotary_cos"), py::arg("rotary_sin"), py::arg("cache_batch_idx"),
          py::arg("block_table"), py::arg("alibi_slopes"), py::arg("out"),
          py::arg("softmax_scale"), py::arg("is_causal"), py::arg("window_size_left"),
          py::arg("window_size_right"), py::arg("softcap"), py::arg("is_rotary_interleaved"),
          py::arg("num_splits"), py::arg("cache_leftpad") = py::none());
    m.def("bwd", &mha_bwd, "Backward pass");
    m.def("varlen_bwd", &mha_varlen_bwd, "Backward pass (variable length)");
    m.def("fwd_kvcache_fp8", &mha_fwd_kvcache_fp8, "Paged decode over an fp8 e4m3fn K/V cache");
    m.def("fwd_fp8", &mha_fwd_fp8, "Forward pass over fp8 e4m3fn q/k/v (fp8 MFMA)");
    m.def("version", []() { return std::string(fmha_version()); });
}
