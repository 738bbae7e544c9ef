// qs_policy_api.hip -- the C ABI (include/quadswarm.h) over the policy kernels: the rollout's fused attention
// encoders (qs_policy.h, qs_policy_x3.h) and the PPO update's encoder forward / backward, weight gradients and column
// statistics (qs_policy_train.h).  Its own translation unit: the env step kernels (qs_step.hip) and these build and
// rebuild independently into the same libquadswarm.so.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "quadswarm.h"
#include "qs_common.h"
#include "qs_policy_train.h"
#include "qs_policy.h"
#include "qs_policy_x3.h"
#include "qs_error.h"

static int fail(int code, const std::string& msg) { return qs_fail(code, msg); }
#define QS_HIP(call) QS_HIP_CHECK(call)

#ifdef QS_STAMPS
// the policy kernels' phase stamps (this translation unit's copy of qs_dbg_stamps; tools/policy_stamps.py)
extern "C" int qs_debug_stamps_policy(uint64_t* host, size_t n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(qs::qs_dbg_stamps), n * sizeof(uint64_t)) == hipSuccess ? 0 : -3;
}
#endif

// fused attention-encoder forward (qs_policy.h)
static int attn_check(int32_t B, int32_t K, int32_t H, const qs_attn_tower* towers, int32_t n_towers) {
    if (!towers) return fail(QS_E_INVALID, "NULL towers");
    if (n_towers < 1 || n_towers > QS_ATTN_MAX_TOWERS) return fail(QS_E_INVALID, "n_towers must be 1 or 2");
    if (H != 128 && H != 256) return fail(QS_E_INVALID, "attention hidden size must be 128 or 256");
    if (K < 1 || K > qs::pol::MROWS) return fail(QS_E_INVALID, "neighbours per agent must be 1..64");
    if (B < 1) return fail(QS_E_INVALID, "B must be >= 1");
    if ((long long)B * K * H >= (1ll << 31)) return fail(QS_E_INVALID, "B * K * H must stay below 2^31");
    return QS_OK;
}
template <int H>
static int attn_launch(bool embed, const float* obs, int32_t stride, int32_t so, int32_t off, int32_t B, int32_t K,
                       int32_t nd, const qs::pol::Towers& tw, int32_t n_towers, hipStream_t st, bool x3 = false) {
    const int mu = (qs::pol::MROWS / K) * K;
    const dim3 grid((unsigned)(((long long)B * K + mu - 1) / mu), (unsigned)n_towers), block(qs::pol::NTHR);
    if (x3) {   // the split-f16 contraction (qs_policy_x3.h)
        if (embed) {
            const size_t lds = qs::pol::embed_x3_lds_bytes<H>();
            QS_HIP(hipFuncSetAttribute((const void*)qs::pol::attn_embed_x3_kernel<H>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            hipLaunchKernelGGL(qs::pol::attn_embed_x3_kernel<H>, grid, block, lds, st, obs, stride, so, off, B, K, nd, tw);
        } else {
            const size_t lds = qs::pol::pool_x3_lds_bytes<H>();
            QS_HIP(hipFuncSetAttribute((const void*)qs::pol::attn_pool_x3_kernel<H>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            hipLaunchKernelGGL(qs::pol::attn_pool_x3_kernel<H>, grid, block, lds, st, B, K, tw);
        }
        QS_HIP(hipGetLastError());
        return QS_OK;
    }
    if (embed) {
        const size_t lds = qs::pol::embed_lds_bytes<H>();
        QS_HIP(hipFuncSetAttribute((const void*)qs::pol::attn_embed_kernel<H>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(qs::pol::attn_embed_kernel<H>, grid, block, lds, st, obs, stride, so, off, B, K, nd, tw);
    } else {
        const size_t lds = qs::pol::pool_lds_bytes<H>();
        QS_HIP(hipFuncSetAttribute((const void*)qs::pol::attn_pool_kernel<H>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(qs::pol::attn_pool_kernel<H>, grid, block, lds, st, B, K, tw);
    }
    QS_HIP(hipGetLastError());
    return QS_OK;
}
static int attn_embed_impl(const float* obs, int32_t obs_stride, int32_t self_dim, int32_t nbr_off, int32_t B,
                           int32_t K, int32_t nd, int32_t H, const qs_attn_tower* towers, int32_t n_towers,
                           void* stream, bool x3) {
    int rc = attn_check(B, K, H, towers, n_towers);
    if (rc) return rc;
    if (!obs) return fail(QS_E_INVALID, "NULL obs");
    if (nd < 1 || nd > qs::pol::MAX_ND) return fail(QS_E_INVALID, "features per neighbour must be 1..16");
    if (self_dim < 1 || self_dim > obs_stride) return fail(QS_E_INVALID, "self features must lie inside the obs row");
    if (nd + self_dim > qs::pol::KD0) return fail(QS_E_INVALID, "self + neighbour features must be <= 32");
    if (nbr_off < 0 || nbr_off + K * nd > obs_stride) return fail(QS_E_INVALID, "neighbour block outside the obs row");
    qs::pol::Towers tw{};
    for (int i = 0; i < n_towers; ++i) {
        const qs_attn_tower& t = towers[i];
        if (!t.w_e1p || !t.b_e1 || !t.w_e2p || !t.b_e2 || !t.e2 || !t.e_mean)
            return fail(QS_E_INVALID, "NULL stage-1 tower pointer");
        tw.t[i] = t;
    }
    hipStream_t st = (hipStream_t)stream;
    return H == 256 ? attn_launch<256>(true, obs, obs_stride, self_dim, nbr_off, B, K, nd, tw, n_towers, st, x3)
                    : attn_launch<128>(true, obs, obs_stride, self_dim, nbr_off, B, K, nd, tw, n_towers, st, x3);
}
extern "C" int qs_attn_embed(const float* obs, int32_t obs_stride, int32_t self_dim, int32_t nbr_off, int32_t B,
                             int32_t K, int32_t nd, int32_t H, const qs_attn_tower* towers, int32_t n_towers,
                             void* stream) {
    return attn_embed_impl(obs, obs_stride, self_dim, nbr_off, B, K, nd, H, towers, n_towers, stream, false);
}
extern "C" int qs_attn_embed_x3(const float* obs, int32_t obs_stride, int32_t self_dim, int32_t nbr_off, int32_t B,
                                int32_t K, int32_t nd, int32_t H, const qs_attn_tower* towers, int32_t n_towers,
                                void* stream) {
    return attn_embed_impl(obs, obs_stride, self_dim, nbr_off, B, K, nd, H, towers, n_towers, stream, true);
}
static int attn_pool_impl(int32_t B, int32_t K, int32_t H, const qs_attn_tower* towers, int32_t n_towers,
                          void* stream, bool x3) {
    int rc = attn_check(B, K, H, towers, n_towers);
    if (rc) return rc;
    qs::pol::Towers tw{};
    for (int i = 0; i < n_towers; ++i) {
        const qs_attn_tower& t = towers[i];
        if (!t.e2 || !t.P || !t.w_v1p || !t.b_v1 || !t.w_v2p || !t.b_v2 || !t.w_a1ep || !t.w_a2p || !t.b_a2 ||
            !t.w_a3 || !t.out)
            return fail(QS_E_INVALID, "NULL stage-2 tower pointer");
        tw.t[i] = t;
    }
    return H == 256 ? attn_launch<256>(false, nullptr, 0, 0, 0, B, K, 0, tw, n_towers, (hipStream_t)stream, x3)
                    : attn_launch<128>(false, nullptr, 0, 0, 0, B, K, 0, tw, n_towers, (hipStream_t)stream, x3);
}
extern "C" int qs_attn_pool(int32_t B, int32_t K, int32_t H, const qs_attn_tower* towers, int32_t n_towers,
                            void* stream) {
    return attn_pool_impl(B, K, H, towers, n_towers, stream, false);
}
extern "C" int qs_attn_pool_x3(int32_t B, int32_t K, int32_t H, const qs_attn_tower* towers, int32_t n_towers,
                               void* stream) {
    return attn_pool_impl(B, K, H, towers, n_towers, stream, true);
}

// the PPO update's attention encoder (qs_policy_train.h)
enum { TR_EMBED, TR_POOL, TR_BWD1, TR_BWD2 };
template <int H>
static int attn_train_launch(int what, const float* obs, int32_t stride, int32_t so, int32_t off, int32_t B, int32_t K,
                             int32_t nd, const qs::pol::Towers& tw, const qs::pol::Trains& trs, int32_t n_towers,
                             hipStream_t st) {
    namespace P = qs::pol;
    const int mu = (P::MROWS / K) * K;
    const dim3 grid((unsigned)(((long long)B * K + mu - 1) / mu), (unsigned)n_towers), block(P::NTHR);
    size_t lds = 0;
    const void* fn = nullptr;
    switch (what) {
        case TR_EMBED: lds = P::embed_x3_lds_bytes<H>(); fn = (const void*)P::attn_embed_train_x3_kernel<H>; break;
        case TR_POOL: lds = P::pool_x3_lds_bytes<H>(); fn = (const void*)P::attn_pool_train_x3_kernel<H>; break;
        case TR_BWD1: lds = P::bwd1_lds_bytes<H>(K); fn = (const void*)P::attn_bwd1_x3_kernel<H>; break;
        default: lds = P::bwd2_lds_bytes<H>(); fn = (const void*)P::attn_bwd2_x3_kernel<H>; break;
    }
    QS_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    switch (what) {
        case TR_EMBED:
            hipLaunchKernelGGL(P::attn_embed_train_x3_kernel<H>, grid, block, lds, st, obs, stride, so, off, B, K, nd, tw, trs);
            break;
        case TR_POOL: hipLaunchKernelGGL(P::attn_pool_train_x3_kernel<H>, grid, block, lds, st, B, K, tw, trs); break;
        case TR_BWD1: hipLaunchKernelGGL(P::attn_bwd1_x3_kernel<H>, grid, block, lds, st, B, K, tw, trs); break;
        default: hipLaunchKernelGGL(P::attn_bwd2_x3_kernel<H>, grid, block, lds, st, B, K, tw, trs); break;
    }
    QS_HIP(hipGetLastError());
    return QS_OK;
}
static int attn_train_impl(int what, const float* obs, int32_t stride, int32_t so, int32_t off, int32_t B, int32_t K,
                           int32_t nd, int32_t H, const qs_attn_tower* towers, const qs_attn_train* trains,
                           int32_t n_towers, void* stream) {
    int rc = attn_check(B, K, H, towers, n_towers);
    if (rc) return rc;
    if (!trains) return fail(QS_E_INVALID, "NULL trains");
    if (what == TR_EMBED) {
        if (!obs) return fail(QS_E_INVALID, "NULL obs");
        if (nd < 1 || nd > qs::pol::MAX_ND) return fail(QS_E_INVALID, "features per neighbour must be 1..16");
        if (so < 1 || so > stride) return fail(QS_E_INVALID, "self features must lie inside the obs row");
        if (nd + so > qs::pol::KD0) return fail(QS_E_INVALID, "self + neighbour features must be <= 32");
        if (off < 0 || off + K * nd > stride) return fail(QS_E_INVALID, "neighbour block outside the obs row");
    }
    qs::pol::Towers tw{};
    qs::pol::Trains trs{};
    for (int i = 0; i < n_towers; ++i) {
        const qs_attn_tower& t = towers[i];
        const qs_attn_train& r = trains[i];
        bool ok = true;
        switch (what) {
            case TR_EMBED: ok = t.w_e1p && t.b_e1 && t.w_e2p && t.b_e2 && t.e2 && t.e_mean && r.e1; break;
            case TR_POOL:
                ok = t.e2 && t.P && t.w_v1p && t.b_v1 && t.w_v2p && t.b_v2 && t.w_a1ep && t.w_a2p && t.b_a2 && t.w_a3 &&
                     t.out && r.a1 && r.a2 && r.v1 && r.h && r.w;
                break;
            case TR_BWD1:
                ok = t.w_a3 && r.w && r.h && r.v1 && r.a1 && r.a2 && r.dout && r.w_v2tp && r.w_v1tp && r.w_a2tp &&
                     r.w_a1etp && r.dh_pre && r.dv1_pre && r.da2_pre && r.da1_pre && r.dscore && r.de2p;
                break;
            default: ok = t.e2 && r.e1 && r.de2p && r.dem && r.w_e2tp && r.de2_pre && r.de1_pre; break;
        }
        if (!ok) return fail(QS_E_INVALID, "NULL tower / train pointer for this stage");
        tw.t[i] = t;
        trs.t[i] = r;
    }
    hipStream_t st = (hipStream_t)stream;
    return H == 256 ? attn_train_launch<256>(what, obs, stride, so, off, B, K, nd, tw, trs, n_towers, st)
                    : attn_train_launch<128>(what, obs, stride, so, off, B, K, nd, tw, trs, n_towers, st);
}
extern "C" int qs_attn_embed_train_x3(const float* obs, int32_t obs_stride, int32_t self_dim, int32_t nbr_off, int32_t B,
                                      int32_t K, int32_t nd, int32_t H, const qs_attn_tower* towers,
                                      const qs_attn_train* trains, int32_t n_towers, void* stream) {
    return attn_train_impl(TR_EMBED, obs, obs_stride, self_dim, nbr_off, B, K, nd, H, towers, trains, n_towers, stream);
}
extern "C" int qs_attn_pool_train_x3(int32_t B, int32_t K, int32_t H, const qs_attn_tower* towers,
                                     const qs_attn_train* trains, int32_t n_towers, void* stream) {
    return attn_train_impl(TR_POOL, nullptr, 0, 0, 0, B, K, 0, H, towers, trains, n_towers, stream);
}
extern "C" int qs_attn_bwd1_x3(int32_t B, int32_t K, int32_t H, const qs_attn_tower* towers,
                               const qs_attn_train* trains, int32_t n_towers, void* stream) {
    return attn_train_impl(TR_BWD1, nullptr, 0, 0, 0, B, K, 0, H, towers, trains, n_towers, stream);
}
template <int H>
static int dw_launch(const float* G, int32_t ldg, const float* A, int32_t lda, const float* gs, int64_t R, float* part,
                     float* part_sum, int32_t n_parts, hipStream_t st) {
    namespace P = qs::pol;
    const long long rows_per = (R + n_parts - 1) / n_parts;
    const int steps = (int)((rows_per + P::DW_STEP - 1) / P::DW_STEP);
    const size_t lds = P::dw_lds_bytes<H>();
    QS_HIP(hipFuncSetAttribute((const void*)P::dw_x3_kernel<H>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    if ((long long)steps * P::DW_STEP * (ldg > lda ? ldg : lda) * 4 >= (1ll << 31))
        return fail(QS_E_INVALID, "rows per part x row stride too large (use more parts)");
    hipLaunchKernelGGL(P::dw_x3_kernel<H>, dim3((unsigned)n_parts), dim3(P::dw_threads<H>()), lds, st, G, A, gs, (long)R, steps, part,
                       part_sum, (int)ldg, (int)lda);
    QS_HIP(hipGetLastError());
    return QS_OK;
}
extern "C" int qs_dw_x3_ld(const float* G, int32_t ldg, const float* A, int32_t lda, const float* col_scale, int64_t R,
                           int32_t H, float* part, float* part_sum, int32_t n_parts, void* stream) {
    if (!G || !A || !col_scale || !part) return fail(QS_E_INVALID, "NULL argument");
    if (H != 128 && H != 256) return fail(QS_E_INVALID, "hidden size must be 128 or 256");
    if (ldg < H || lda < H || ldg > 4096 || lda > 4096) return fail(QS_E_INVALID, "row strides H .. 4096 floats");
    if (R < 1 || n_parts < 1 || n_parts > 65535 || R * (int64_t)(ldg > lda ? ldg : lda) >= (1ll << 40))
        return fail(QS_E_INVALID, "R >= 1, 1 <= n_parts <= 65535");
    hipStream_t st = (hipStream_t)stream;
    return H == 256 ? dw_launch<256>(G, ldg, A, lda, col_scale, R, part, part_sum, n_parts, st)
                    : dw_launch<128>(G, ldg, A, lda, col_scale, R, part, part_sum, n_parts, st);
}
extern "C" int qs_attn_dw_x3(const float* G, const float* A, const float* col_scale, int64_t R, int32_t H, float* part,
                             float* part_sum, int32_t n_parts, void* stream) {
    return qs_dw_x3_ld(G, H, A, H, col_scale, R, H, part, part_sum, n_parts, stream);
}
template <int H>
static int dw0_launch(const float* G, const float* gs, const float* obs, int32_t stride, int32_t so, int32_t off,
                      int32_t B, int32_t K, int32_t nd, float* part, float* part_sum, int32_t n_parts, hipStream_t st) {
    namespace P = qs::pol;
    const long long R = (long long)B * K;
    const long long rows_per = (R + n_parts - 1) / n_parts;
    const int steps = (int)((rows_per + P::DW_STEP - 1) / P::DW_STEP);
    const size_t lds = P::dw0_lds_bytes<H>();
    QS_HIP(hipFuncSetAttribute((const void*)P::dw0_x3_kernel<H>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(P::dw0_x3_kernel<H>, dim3((unsigned)n_parts), dim3(P::NTHR), lds, st, G, gs, obs, stride, so, off,
                       B, K, nd, (long)R, steps, part, part_sum);
    QS_HIP(hipGetLastError());
    return QS_OK;
}
extern "C" int qs_attn_dw0_x3(const float* G, const float* col_scale, const float* obs, int32_t stride, int32_t so,
                              int32_t off, int32_t B, int32_t K, int32_t nd, int32_t H, float* part, float* part_sum,
                              int32_t n_parts, void* stream) {
    namespace P = qs::pol;
    if (!G || !col_scale || !obs || !part) return fail(QS_E_INVALID, "NULL argument");
    if (H != 128 && H != 256) return fail(QS_E_INVALID, "hidden size must be 128 or 256");
    if (B < 1 || K < 1 || (int64_t)B * K >= (1ll << 31) || n_parts < 1 || n_parts > 65535)
        return fail(QS_E_INVALID, "B, K >= 1, B K < 2^31, 1 <= n_parts <= 65535");
    if (nd < 0 || so < 1 || nd + so > P::KD0) return fail(QS_E_INVALID, "nd >= 0, self_dim >= 1, nd + self_dim <= 32");
    if (so > stride || off < 0 || off + (int64_t)K * nd > stride)
        return fail(QS_E_INVALID, "self features and the neighbour block must lie inside the obs row");
    hipStream_t st = (hipStream_t)stream;
    return H == 256 ? dw0_launch<256>(G, col_scale, obs, stride, so, off, B, K, nd, part, part_sum, n_parts, st)
                    : dw0_launch<128>(G, col_scale, obs, stride, so, off, B, K, nd, part, part_sum, n_parts, st);
}
extern "C" int qs_linear_tanh_x3(const float* X, int64_t M, int32_t K, const void* w_packed, int64_t w_bytes,
                                 const float* bias, float* Y, int32_t N, void* stream) {
    namespace P = qs::pol;
    if (!X || !w_packed || !bias || !Y) return fail(QS_E_INVALID, "NULL argument");
    if (M < 1 || M >= (1ll << 31) / 512 || (K != 256 && K != 512) || N < 256 || N > 1024 || N % 256)
        return fail(QS_E_INVALID, "M >= 1, K 256 or 512, N a multiple of 256 up to 1024");
    // the packed operand: (N / 256) (K / 256) blocks of 256 x 256 weights as f16 hi + lo halves
    if (w_bytes != (int64_t)(N / 256) * (K / 256) * 256 * 256 * 2 * 2)
        return fail(QS_E_INVALID, "w_bytes: the packed weight must hold (N / 256) (K / 256) packed 256 x 256 blocks");
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)((M + P::MROWS - 1) / P::MROWS), (unsigned)(N / 256));
    const size_t lds = P::linear_x3_lds_bytes();
    const uint4* wp = reinterpret_cast<const uint4*>(w_packed);
    if (K == 256) {
        QS_HIP(hipFuncSetAttribute((const void*)P::linear_tanh_x3_kernel<1, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL((P::linear_tanh_x3_kernel<1, false, true>), grid, dim3(P::NTHR), lds, st, X, X + 256, (long)K, (long)M, wp, bias, Y, N,
                           nullptr);
    } else {
        QS_HIP(hipFuncSetAttribute((const void*)P::linear_tanh_x3_kernel<2, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL((P::linear_tanh_x3_kernel<2, false, true>), grid, dim3(P::NTHR), lds, st, X, X + 256, (long)K, (long)M, wp, bias, Y, N,
                           nullptr);
    }
    QS_HIP(hipGetLastError());
    return QS_OK;
}
extern "C" int qs_linear_tanh_cat_x3(const float* X0, const float* X1, int64_t M, const void* w_packed, int64_t w_bytes,
                                     const float* bias, float* Y, int32_t N, void* stream) {
    namespace P = qs::pol;
    if (!X0 || !X1 || !w_packed || !bias || !Y) return fail(QS_E_INVALID, "NULL argument");
    if (M < 1 || M >= (1ll << 31) / 512 || N < 256 || N > 1024 || N % 256)
        return fail(QS_E_INVALID, "M >= 1, N a multiple of 256 up to 1024");
    if (w_bytes != (int64_t)(N / 256) * 2 * 256 * 256 * 2 * 2)
        return fail(QS_E_INVALID, "w_bytes: the packed weight must hold (N / 256) 2 packed 256 x 256 blocks");
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)((M + P::MROWS - 1) / P::MROWS), (unsigned)(N / 256));
    const size_t lds = P::linear_x3_lds_bytes();
    QS_HIP(hipFuncSetAttribute((const void*)P::linear_tanh_x3_kernel<2, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL((P::linear_tanh_x3_kernel<2, false, true>), grid, dim3(P::NTHR), lds, st, X0, X1, 256l, (long)M,
                       reinterpret_cast<const uint4*>(w_packed), bias, Y, N, nullptr);
    QS_HIP(hipGetLastError());
    return QS_OK;
}
extern "C" int qs_linear_rows_x3(const float* X, const float* row_scale, int64_t M, int32_t K, const void* w_packed,
                                 int64_t w_bytes, float* Y, int32_t N, void* stream) {
    namespace P = qs::pol;
    if (!X || !row_scale || !w_packed || !Y) return fail(QS_E_INVALID, "NULL argument");
    if (M < 1 || M >= (1ll << 31) / 512 || (K != 256 && K != 512) || N < 256 || N > 1024 || N % 256)
        return fail(QS_E_INVALID, "M >= 1, K 256 or 512, N a multiple of 256 up to 1024");
    if (w_bytes != (int64_t)(N / 256) * (K / 256) * 256 * 256 * 2 * 2)
        return fail(QS_E_INVALID, "w_bytes: the packed weight must hold (N / 256) (K / 256) packed 256 x 256 blocks");
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)((M + P::MROWS - 1) / P::MROWS), (unsigned)(N / 256));
    const size_t lds = P::linear_x3_lds_bytes();
    const uint4* wp = reinterpret_cast<const uint4*>(w_packed);
    if (K == 256) {
        QS_HIP(hipFuncSetAttribute((const void*)P::linear_tanh_x3_kernel<1, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL((P::linear_tanh_x3_kernel<1, true, true>), grid, dim3(P::NTHR), lds, st, X, X + 256, (long)K, (long)M, wp, nullptr, Y, N,
                           row_scale);
    } else {
        QS_HIP(hipFuncSetAttribute((const void*)P::linear_tanh_x3_kernel<2, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL((P::linear_tanh_x3_kernel<2, true, true>), grid, dim3(P::NTHR), lds, st, X, X + 256, (long)K, (long)M, wp, nullptr, Y, N,
                           row_scale);
    }
    QS_HIP(hipGetLastError());
    return QS_OK;
}
extern "C" int qs_tanh_grad_stats(const float* g, const float* y, float* gp, float* row_scale, float* col_part, int64_t M,
                                  int32_t N, void* stream) {
    namespace P = qs::pol;
    if (!g || !y || !gp || !row_scale || !col_part) return fail(QS_E_INVALID, "NULL argument");
    if (M < 1 || M >= (1ll << 31) / 512 || (N != 256 && N != 512)) return fail(QS_E_INVALID, "M >= 1, N 256 or 512");
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)((M + P::MROWS - 1) / P::MROWS));
    if (N == 256)
        hipLaunchKernelGGL(P::tanh_grad_stats_kernel<1>, grid, dim3(P::NTHR), 0, st, g, y, gp, row_scale, col_part, (long)M);
    else
        hipLaunchKernelGGL(P::tanh_grad_stats_kernel<2>, grid, dim3(P::NTHR), 0, st, g, y, gp, row_scale, col_part, (long)M);
    QS_HIP(hipGetLastError());
    return QS_OK;
}
extern "C" int qs_linear_bias_x3(const float* X, int64_t M, int32_t K, const void* w_packed, int64_t w_bytes,
                                 const float* bias, float* Y, int32_t N, void* stream) {
    namespace P = qs::pol;
    if (!X || !w_packed || !bias || !Y) return fail(QS_E_INVALID, "NULL argument");
    if (M < 1 || M >= (1ll << 31) / 512 || (K != 256 && K != 512) || N < 256 || N > 1024 || N % 256)
        return fail(QS_E_INVALID, "M >= 1, K 256 or 512, N a multiple of 256 up to 1024");
    if (w_bytes != (int64_t)(N / 256) * (K / 256) * 256 * 256 * 2 * 2)
        return fail(QS_E_INVALID, "w_bytes: the packed weight must hold (N / 256) (K / 256) packed 256 x 256 blocks");
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)((M + P::MROWS - 1) / P::MROWS), (unsigned)(N / 256));
    const size_t lds = P::linear_x3_lds_bytes();
    const uint4* wp = reinterpret_cast<const uint4*>(w_packed);
    if (K == 256) {
        QS_HIP(hipFuncSetAttribute((const void*)P::linear_tanh_x3_kernel<1, false, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL((P::linear_tanh_x3_kernel<1, false, false>), grid, dim3(P::NTHR), lds, st, X, X + 256, (long)K, (long)M, wp, bias, Y,
                           N, nullptr);
    } else {
        QS_HIP(hipFuncSetAttribute((const void*)P::linear_tanh_x3_kernel<2, false, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL((P::linear_tanh_x3_kernel<2, false, false>), grid, dim3(P::NTHR), lds, st, X, X + 256, (long)K, (long)M, wp, bias, Y,
                           N, nullptr);
    }
    QS_HIP(hipGetLastError());
    return QS_OK;
}
extern "C" int qs_slab_sum_stats(const float* G, int32_t n_slabs, int64_t M, int32_t N, float* out, float* row_scale,
                                 float* col_part, void* stream) {
    namespace P = qs::pol;
    if (!G || !out || !row_scale || !col_part) return fail(QS_E_INVALID, "NULL argument");
    if (n_slabs < 1 || M < 1 || (int64_t)n_slabs * M >= (1ll << 31) / 512 || (N != 256 && N != 512))
        return fail(QS_E_INVALID, "n_slabs >= 1, M >= 1, n_slabs M < 2^22, N 256 or 512");
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)((M + P::MROWS - 1) / P::MROWS));
    if (N == 256)
        hipLaunchKernelGGL(P::slab_sum_stats_kernel<1>, grid, dim3(P::NTHR), 0, st, G, (int)n_slabs, out, row_scale, col_part,
                           (long)M);
    else
        hipLaunchKernelGGL(P::slab_sum_stats_kernel<2>, grid, dim3(P::NTHR), 0, st, G, (int)n_slabs, out, row_scale, col_part,
                           (long)M);
    QS_HIP(hipGetLastError());
    return QS_OK;
}
extern "C" int qs_colmax_reduce(const float* part_max, int32_t n_stats, int32_t n_blocks, int32_t H, float* out,
                                void* stream) {
    namespace P = qs::pol;
    if (!part_max || !out) return fail(QS_E_INVALID, "NULL argument");
    if (n_stats < 1 || n_stats > QS_ATTN_NCOLMAX || n_blocks < 1 || H < 1 || H > 4096)
        return fail(QS_E_INVALID, "1 <= n_stats <= QS_ATTN_NCOLMAX, n_blocks >= 1, 1 <= H <= 4096");
    hipStream_t st = (hipStream_t)stream;
    QS_HIP(hipMemsetAsync(out, 0, (size_t)n_stats * H * sizeof(float), st));
    hipLaunchKernelGGL(P::colmax_reduce_kernel, dim3(P::CM_CHUNKS, (unsigned)((H + 63) / 64), (unsigned)n_stats),
                       dim3(256), 0, st, part_max, n_blocks, H, out);
    QS_HIP(hipGetLastError());
    return QS_OK;
}
extern "C" int qs_colstats(const float* G, int64_t R, int32_t H, const float* row_w, const float* obs, int32_t stride,
                           int32_t nbr_off, int32_t B, int32_t K, int32_t nd, int32_t nx, float* pmx, float* psm,
                           float* px, int32_t n_parts, void* stream) {
    namespace P = qs::pol;
    if (!G || !pmx || !psm) return fail(QS_E_INVALID, "NULL argument");
    if (H != 128 && H != 256) return fail(QS_E_INVALID, "hidden size must be 128 or 256");
    if (R < 1 || n_parts < 1 || n_parts > (1 << 24) || R * (int64_t)H >= (1ll << 40))
        return fail(QS_E_INVALID, "R >= 1, 1 <= n_parts <= 2^24");
    if (nx < 0 || nx > QS_COLSTATS_MAX_X) return fail(QS_E_INVALID, "nx out of range");
    if (nx > 0 && (!obs || !px || B < 1 || K < 1 || nd < 0 || nd > nx || (int64_t)B * K != R || R >= (1ll << 31) ||
                   stride < nx ||
                   nbr_off < 0 || nbr_off + (int64_t)K * nd > stride))
        return fail(QS_E_INVALID, "layer-0 input: obs, part_x, B K = R, nd <= nx, the neighbour block inside a row");
    hipStream_t st = (hipStream_t)stream;
    const long rows_per = (long)((R + n_parts - 1) / n_parts);
    if (nx > 8)
        hipLaunchKernelGGL(P::colstats_kernel<QS_COLSTATS_MAX_X>, dim3((unsigned)n_parts), dim3(H), 0, st, G, (long)R, H,
                           rows_per, row_w, obs, stride, nbr_off, B, K, nd, nx, pmx, psm, px);
    else if (nx > 0)   // the neighbour features alone (nd <= 8)
        hipLaunchKernelGGL(P::colstats_kernel<8>, dim3((unsigned)n_parts), dim3(H), 0, st, G, (long)R, H, rows_per, row_w,
                           obs, stride, nbr_off, B, K, nd, nx, pmx, psm, px);
    else
        hipLaunchKernelGGL(P::colstats_kernel<0>, dim3((unsigned)n_parts), dim3(H), 0, st, G, (long)R, H, rows_per,
                           row_w, obs, stride, nbr_off, B > 0 ? B : 1, K > 0 ? K : 1, nd, 0, pmx, psm, px);
    QS_HIP(hipGetLastError());
    return QS_OK;
}
extern "C" int qs_attn_bwd2_x3(int32_t B, int32_t K, int32_t H, const qs_attn_tower* towers,
                               const qs_attn_train* trains, int32_t n_towers, void* stream) {
    return attn_train_impl(TR_BWD2, nullptr, 0, 0, 0, B, K, 0, H, towers, trains, n_towers, stream);
}

