// Blocked stage 1: the read passes k_rpass (Y = A^T V, X = A U, split-K on the
// matrix cores) and the virtual tile's partial sum k_vsum (gfx950).
#include "brd_blk.h"

#include <cstdlib>

namespace brd {
namespace blk {

// ==========================================================================
// k_rpass: D = B^T S (Y pass) or S B (X pass) for a tall "skinny" operand B
// (K x 32) and a source S, summed over one split of the K range.
//   Y pass (YP): S(k, m) = src[k*ld + m] (row-major A, k = rows, m = columns),
//                D[t][m] = sum_k B[k][t] S(k, m); partials stored [split][t][m].
//   X pass     : S(k, m) = src[m*ld + k] (k = columns, m = rows),
//                D[m][t] = sum_k S(k, m) B[k][t]; partials stored [split][m][t].
// B(k, t) = bsrc[k*bld + t] in both.  Every wave streams its own 64 values of
// m straight from HBM into MFMA operand registers (no LDS, no barriers):
//   Y: one 16-byte load per lane and 4 rows gives 2 x 16 columns (even / odd
//      column tiles), 4 rows x 256 contiguous bytes per instruction;
//   X: one 16-byte load per lane gives 2 k of one row: 16 rows x 64 bytes per
//      instruction, two K steps each;
// with kSU steps of loads in flight (static register ring).  The "virtual"
// workgroups (the first ksplit of the grid) compute the same product with
// S = vsrc (256 wide); they meet at a counter and each sums one slice of
// their partials into vout in fixed order (deterministic).
// ==========================================================================
template <typename T, bool YP, typename FA>
__global__ void __launch_bounds__(kRT, 1) k_rpass(RpArgs a, FA fin) {
    typedef typename G2<T>::v2 v2;
    typedef typename Mf<T>::v4 v4;
    const int tid = threadIdx.x, lane = tid & 63, w = (tid >> 6) & 3, kh = tid >> 8;
    const int q = lane >> 4, l15 = lane & 15;
    // one LDS block for the K halves' reduction and (workgroup 0) cqr_finish:
    // 64 KB, so two workgroups share a CU
    __shared__ __attribute__((aligned(16))) double rp_lds[kRpLds];
    if (a.has_fin && blockIdx.x == 0) {   // the previous panel's LU, T and R signs, beside the pass
        cqr_finish_entry<T>(fin, tid, rp_lds);
        return;
    }
    const int bid = blockIdx.x - a.has_fin;
    const bool virt = bid < a.nvirt;
    int mx, ks;
    if (virt) { mx = 0; ks = bid; }
    else      { const int r = bid - a.nvirt; mx = r % a.mtiles; ks = r / a.mtiles; }
    const T *S;
    long ld;
    int M;
    if (virt) { S = (const T *)a.vsrc; ld = a.vld; M = kMT; }
    else      { S = (const T *)a.src + (YP ? (long)mx * kMT : (long)mx * kMT * a.ld); ld = a.ld; M = min(kMT, a.M - mx * kMT); }
    const T *B = (const T *)a.bsrc;
    // waves w and w + 4 take the two halves of the workgroup's K range (in
    // whole 8-row step pairs) and meet in LDS: two waves per SIMD in flight
    const int kb0 = ks * a.kper, ke0 = min(a.K, kb0 + a.kper);
    const int khalf = ke0 > kb0 ? ((ke0 - kb0 + 15) / 16) * 8 : 0;
    const int kbeg = kh ? min(ke0, kb0 + khalf) : kb0, kend = kh ? ke0 : min(ke0, kb0 + khalf);
    const int mb = kWM * w;
    v4 acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = v4{0, 0, 0, 0};

    if constexpr (YP) {
        // acc[h*4 + p*2 + e]: t-half h, column pair group p (32 columns), parity e
        const int nst = kend > kbeg ? (kend - kbeg + 3) / 4 : 0;
        v2 ra[kSU][2];
        T rb[kSU][2];
        auto load = [&](int s, v2 (&va)[2], T (&vb)[2]) {
            const int k = kbeg + 4 * s + q;
            const bool kv = k < kend;
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                const int m = mb + 32 * p + 2 * l15;
                v2 v = {(T)0, (T)0};
                if (kv && m < M) {
                    const T *src = S + (long)k * ld + m;
                    if (m + 1 < M) v = *(const v2 *)src; else v.x = src[0];
                }
                va[p] = v;
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) vb[h] = kv ? B[(long)k * a.bld + 16 * h + l15] : (T)0;
        };
#pragma unroll
        for (int u = 0; u < kSU; ++u)
            if (u < nst) load(u, ra[u], rb[u]);
        for (int s0 = 0; s0 < nst; s0 += kSU) {
#pragma unroll
            for (int u = 0; u < kSU; ++u) {
                const int s = s0 + u;
                if (s < nst) {
#pragma unroll
                    for (int h = 0; h < 2; ++h)
#pragma unroll
                        for (int p = 0; p < 2; ++p) {
                            acc[h * 4 + p * 2 + 0] = Mf<T>::mma(rb[u][h], ra[u][p].x, acc[h * 4 + p * 2 + 0]);
                            acc[h * 4 + p * 2 + 1] = Mf<T>::mma(rb[u][h], ra[u][p].y, acc[h * 4 + p * 2 + 1]);
                        }
                    if (s + kSU < nst) load(s + kSU, ra[u], rb[u]);
                }
            }
        }
    } else {
        // acc[p*2 + h]: row tile p (16 rows), t-half h; one step pair = 8 k
        const int npr = kend > kbeg ? (kend - kbeg + 7) / 8 : 0;
        constexpr int kSP2 = kSU / 2;
        v2 ra[kSP2][4];
        T rb[kSP2][2][2];
        auto load = [&](int s2, v2 (&va)[4], T (&vb)[2][2]) {
            const int k = kbeg + 8 * s2 + 2 * q;
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const int m = mb + 16 * p + l15;
                v2 v = {(T)0, (T)0};
                if (m < M && k < kend) {
                    const T *src = S + (long)m * ld + k;
                    if (k + 1 < kend) v = *(const v2 *)src; else v.x = src[0];
                }
                va[p] = v;
            }
#pragma unroll
            for (int e = 0; e < 2; ++e)
#pragma unroll
                for (int h = 0; h < 2; ++h) vb[e][h] = (k + e < kend) ? B[(long)(k + e) * a.bld + 16 * h + l15] : (T)0;
        };
#pragma unroll
        for (int u = 0; u < kSP2; ++u)
            if (u < npr) load(u, ra[u], rb[u]);
        for (int s0 = 0; s0 < npr; s0 += kSP2) {
#pragma unroll
            for (int u = 0; u < kSP2; ++u) {
                const int s2 = s0 + u;
                if (s2 < npr) {
#pragma unroll
                    for (int p = 0; p < 4; ++p)
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            acc[p * 2 + h] = Mf<T>::mma(ra[u][p].x, rb[u][0][h], acc[p * 2 + h]);
                            acc[p * 2 + h] = Mf<T>::mma(ra[u][p].y, rb[u][1][h], acc[p * 2 + h]);
                        }
                    if (s2 + kSP2 < npr) load(s2 + kSP2, ra[u], rb[u]);
                }
            }
        }
    }

    // ---- the second half's sums into the first half's, fixed order ----------
    {
        T (*red)[32][64] = reinterpret_cast<T (*)[32][64]>(rp_lds);
        if (kh) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int g = 0; g < 4; ++g) red[w][4 * i + g][lane] = acc[i][g];
        }
        __syncthreads();
        if (!kh) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int g = 0; g < 4; ++g) acc[i][g] += red[w][4 * i + g][lane];
        }
    }
    // ---- partials ----------------------------------------------------------
    T *out;
    long mp;
    if (virt) { out = (T *)a.vpart + (size_t)ks * 32 * kMT; mp = kMT; }
    else      { out = (T *)a.part + (size_t)ks * 32 * a.mp + (size_t)mx * kMT * (YP ? 1 : 32); mp = a.mp; }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            if (kh) break;
            const int r = Mf<T>::crow(q, g);
            if (YP) {
                const int h = i >> 2, p = (i >> 1) & 1, e = i & 1;
                const int t = 16 * h + r, m = mb + 32 * p + 2 * l15 + e;
                if (m < M) out[(size_t)t * mp + m] = acc[i][g];
            } else {
                const int p = i >> 1, h = i & 1;
                const int m = mb + 16 * p + r, t = 16 * h + l15;
                if (m < M) out[(size_t)m * 32 + t] = acc[i][g];
            }
        }
}

// The virtual tile's split-K partials summed in fixed order (one element per
// thread, every partial's load in flight at once): a kernel of its own, so
// no workgroup of the read pass waits for another.
// Workgroup 0 also patches the diagonal of the finished panel's top block
// from V' = Q to V = Q - S (pbase[t (pstride)] -= s_t), read from here on.
template <typename T>
__global__ void __launch_bounds__(256) k_vsum(const T *vpart, T *vout, int nvirt, T *pbase, long pstride,
                                              const double *sgn) {
    const int e = blockIdx.x * 256 + threadIdx.x;   // < 32 kMT
    if (blockIdx.x == 0 && threadIdx.x < 32 && pbase)
        pbase[(size_t)threadIdx.x * pstride] = (T)((double)pbase[(size_t)threadIdx.x * pstride] - sgn[threadIdx.x]);
    T v[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) v[k] = vpart[(size_t)min(k, nvirt - 1) * 32 * kMT + e];
    T s = v[0];
#pragma unroll
    for (int k = 1; k < 32; ++k)
        if (k < nvirt) s += v[k];
    vout[e] = s;
}

// ==========================================================================
// k_rpass_d: the same read passes with the source stream staged through LDS
// by LDS-DMA (k_rpass's X pass loads 16 rows x 64 B per
// wave instruction, and both passes keep only 8 K steps of 16 B per lane in
// flight).  Every DMA instruction moves whole >= 128-B row segments: the Y
// pass 2 KB rows of the 256-column tile (two 1-KB instructions per row), the
// X pass 128-B segments of 8 rows; kRS stages of 16 k (32 KB each) are in
// flight per workgroup, with no staging registers.  The 8 waves share the K
// stream (no K halves to reduce): wave w owns 32 of the tile's 256 m.
//   Y: D[t][m] = sum_k B[k][t] S(k, m), S(k, m) = src[k ld + m]; LDS [k][m]
//      (pitch 272: four k rows in distinct bank halves)
//   X: D[m][t] = sum_k S(k, m) B[k][t], S(k, m) = src[m ld + k]; LDS [m][k]
//      with the k pairs of row m XOR-swizzled by (m >> 1) & 7 (the DMA lane
//      loads the pair that belongs in its slot): a half-wave's 16 rows x 16 B
//      cover the 64 banks once
// B (K x 32) is DMA'd beside it, [k][32], odd k rows with their halves
// swapped (t pairs XOR 8), so rows k and k + 1 read disjoint banks.
// Rows, columns and k past the source read 0 (offset past num_records);
// the host uses this kernel when no 16-byte pair straddles the source's end
// (Y: M even, X: K even -- always, for even n).
// ==========================================================================
#ifndef BRD_RPASS_HOIST
#define BRD_RPASS_HOIST 0   // A/B knob (tools/variant_lib.sh): 1 measured no faster (X pass 110 -> 113 us)
#endif
// stages in the ring (kRS - 1 in flight).  Round 6, N = 8192 fp64 one at a
// time, same box: rings of 2 / 3 / 4 stages 21.45 / 21.25 / 21.72-21.84 ms of
// read passes per matrix, the stream unchanged; the next stage's DMAs spread
// between the MFMA steps 22.7, the source stream non-temporal 21.8 -- the
// large passes are not bound by the bytes in flight or the DMA issue
constexpr int kRS = 4;
// wait until at most `younger` stages' DMAs are outstanding (waves 0-3 issue
// 5 a stage, 4-7 issue 4; vmcnt counts in order)
template <int Y> __device__ __forceinline__ void rp_wait(bool five) {
    if (five) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 * Y) : "memory");
    else      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * Y) : "memory");
}
constexpr int kSY = 272;    // Y stage pitch (elements per k row: rows k..k+3 of a read in distinct banks)
struct RpLdsD {             // 32 KB of source + 4 KB of B per stage, either type
    double s[kRS][16 * kSY];    // Y [k][272]; X [256][kRK]
    double b[kRS][16 * 32];     // [kRK][32]
};
// elements per 16-B vector, k per stage (32 KB of a 256-wide tile)
template <typename T> constexpr int rp_epv() { return 16 / (int)sizeof(T); }
template <typename T> constexpr int rp_krk() { return 128 / (int)sizeof(T); }
// B's t vectors XOR-swizzled per row so the 4 k rows of a read hit distinct banks:
// fp64 rows of 256 B (k, k + 1 in opposite halves), fp32 rows of 128 B (four rows
// in four quarters)
template <typename T> __device__ __forceinline__ int rp_bswz(int k) {
    return sizeof(T) == 8 ? (k & 1) << 3 : ((k >> 1) & 1) << 2;
}

template <typename T, bool YP>
__global__ void __launch_bounds__(kRT, 1) k_rpass_d(RpArgs a, FinArgs fin) {
    static_assert(sizeof(FinLds) <= sizeof(RpLdsD), "cqr_finish's LDS");
    typedef typename Mf<T>::v4 v4;
    constexpr int E = sizeof(T), EPV = rp_epv<T>(), KRK = rp_krk<T>();
    constexpr int BVR = 32 / EPV;            // B: 16-B vectors per row
    constexpr int BRI = 64 / BVR;            // B: rows per DMA instruction
    __shared__ RpLdsD L;
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int q = lane >> 4, l15 = lane & 15;
    if (a.has_fin && blockIdx.x == 0) {   // the previous panel's LU, T and R signs, beside the pass
        cqr_finish_entry<T>(fin, tid, &L);
        return;
    }
    // linearised work: the tiles' KRK-k stages in a row (tile-major; the
    // virtual tile first), wst consecutive stages per workgroup, so every
    // workgroup streams the same bytes whatever the tile count (a workgroup
    // crossing a tile boundary runs two segments).  The contributors of a tile
    // write partial slots 0, 1, ... in k order; its last one zeroes the slots
    // up to ksplit that no workgroup has (fixed-order sums stay deterministic).
    const int g = blockIdx.x - a.has_fin;
    const int tot = a.tiles * a.ns;
    const int uend = min(tot, (g + 1) * a.wst);
    constexpr unsigned kOut = 0x80000000u;
    const unsigned lds_s = (unsigned)(uintptr_t)&L.s[0][0], lds_b = (unsigned)(uintptr_t)&L.b[0][0];
    const T *B = (const T *)a.bsrc;
    const int mb = 32 * w;
    for (int u = g * a.wst; u < uend;) {
        const int tt = u / a.ns, segend = min(uend, (tt + 1) * a.ns);
        const bool virt = a.nvirt > 0 && tt == 0;
        const int mx = tt - (a.nvirt > 0 ? 1 : 0);
        const int slot = g - (tt * a.ns) / a.wst;
        const T *S;
        long ld;
        int M;
        if (virt) { S = (const T *)a.vsrc; ld = a.vld; M = kMT; }
        else      { S = (const T *)a.src + (YP ? (long)mx * kMT : (long)mx * kMT * a.ld); ld = a.ld; M = min(kMT, a.M - mx * kMT); }
        const int kb0 = (u - tt * a.ns) * KRK, ke0 = min(a.K, (segend - tt * a.ns) * KRK);
        const int nst = segend - u;

        // Every wave issues 4 source DMAs (32 per stage) and waves 0-3 one B
        // DMA each; per-lane offsets are relative to the stage's first k (the
        // descriptor's base moves with the stage).
        //   Y: instruction i = 4w + uu covers 1 KB of the stage's rows (fp64:
        //      half a 2-KB row; fp32: a whole 1-KB row)
        //   X: instruction i covers rows 8i..8i+7, 128 B each (lane: row
        //      8i + lane / 8, 16-B slot lane & 7)
        //   B: wave w's instruction covers rows BRI w .. BRI w + BRI - 1
        auto issue_src = [&](int st, int uu) {   // source piece uu (of 4) of stage st
            const int k0 = kb0 + KRK * st, buf = st % kRS;
            if constexpr (YP) {
                const u32x4_t rs = rsrc_of(S + (long)k0 * ld);
                constexpr int IPR = 256 * E / 1024;    // instructions per row
                const int i = 4 * w + uu, kr = i / IPR, h = i % IPR, m = (1024 * h + 16 * lane) / E;
                const unsigned off = (k0 + kr < ke0 && m < M) ? (unsigned)((kr * (int)ld + m) * E) : kOut;
                dma16(rs, off, 0, lds_s + (unsigned)(buf * sizeof(L.s[0]) + (kr * kSY + 1024 / E * h) * E));
            } else {
                const u32x4_t rs = rsrc_of(S + k0);
                const int i = 4 * w + uu, m = 8 * i + (lane >> 3), sl = lane & 7, pr = sl ^ ((m >> 1) & 7);
                const unsigned off = (m < M && k0 + EPV * pr < ke0) ? (unsigned)((m * (int)ld + EPV * pr) * E) : kOut;
                dma16(rs, off, 0, lds_s + (unsigned)(buf * sizeof(L.s[0]) + i * 1024));
            }
        };
        auto issue_b = [&](int st) {   // waves 0-3: their B piece of stage st
            const int k0 = kb0 + KRK * st, buf = st % kRS;
            const u32x4_t rb = rsrc_of(B + (long)k0 * a.bld);
            const int kr = BRI * w + lane / BVR, sl = lane % BVR, tp = sl ^ rp_bswz<T>(kr);
            const unsigned off = k0 + kr < ke0 ? (unsigned)((kr * (int)a.bld + EPV * tp) * E) : kOut;
            dma16(rb, off, 0, lds_b + (unsigned)(buf * sizeof(L.b[0]) + w * 1024));
        };
        auto issue = [&](int st) {
#pragma unroll
            for (int uu = 0; uu < 4; ++uu) issue_src(st, uu);
            if (w < 4) issue_b(st);
        };

        v4 acc[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = v4{(T)0, (T)0, (T)0, (T)0};
#pragma unroll
        for (int st = 0; st < kRS - 1; ++st)
            if (st < nst) issue(st);
        for (int st = 0; st < nst; ++st) {
            // this stage's DMAs landed: the younger stages' (up to kRS - 2) may still fly
            // (in-order vmcnt; waves 0-3 issue 5 DMAs a stage, waves 4-7 issue 4)
            const int younger = min(nst - 1 - st, kRS - 2);
            static_assert(kRS >= 2 && kRS <= 5, "rp_wait cases");
            if (kRS >= 5 && younger >= 3) rp_wait<3>(w < 4);
            else if (kRS >= 4 && younger >= 2) rp_wait<2>(w < 4);
            else if (kRS >= 3 && younger >= 1) rp_wait<1>(w < 4);
            else rp_wait<0>(w < 4);
            __syncthreads();
            // into the buffer every wave finished reading
            if (st + kRS - 1 < nst) issue(st + kRS - 1);
            const int buf = st % kRS;
            const T *ls = (const T *)L.s[buf], *lb = (const T *)L.b[buf];
            // every operand of the stage first (one LDS latency per stage, not
            // one per 4-k step), then the stage's MFMAs back to back
            // (BRD_RPASS_HOIST=1; the default is the per-step form: hoisting
            // measured no faster, profiles/r04_rpass_variants.txt)
            constexpr int NS4 = KRK / 4;
            constexpr int HG = BRD_RPASS_HOIST ? NS4 : 1;   // steps per operand group
#pragma unroll
            for (int s0 = 0; s0 < NS4; s0 += HG) {
                T bt[HG][2], sm[HG][2];
#pragma unroll
                for (int u = 0; u < HG; ++u) {
                    const int k = 4 * (s0 + u) + q;
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int t = 16 * h + l15;
                        bt[u][h] = lb[k * 32 + EPV * ((t / EPV) ^ rp_bswz<T>(k)) + t % EPV];
                    }
#pragma unroll
                    for (int p = 0; p < 2; ++p) {
                        const int m = mb + 16 * p + l15;
                        if constexpr (YP) sm[u][p] = ls[k * kSY + m];
                        else sm[u][p] = ls[m * KRK + EPV * ((k / EPV) ^ ((m >> 1) & 7)) + k % EPV];
                    }
                }
                if constexpr (BRD_RPASS_HOIST) __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead
#pragma unroll
                for (int u = 0; u < HG; ++u)
#pragma unroll
                    for (int i = 0; i < 2; ++i)
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            if constexpr (YP) acc[i][j] = Mf<T>::mma(bt[u][i], sm[u][j], acc[i][j]);   // [t-tile i][m-tile j]
                            else acc[i][j] = Mf<T>::mma(sm[u][i], bt[u][j], acc[i][j]);                // [m-tile i][t-tile j]
                        }
            }
        }
        // ---- partials: slot `slot` of this tile ------------------------------
        T *out;
        long mp, sstride;
        if (virt) { out = (T *)a.vpart; mp = kMT; sstride = 32L * kMT; }
        else      { out = (T *)a.part + (size_t)mx * kMT * (YP ? 1 : 32); mp = a.mp; sstride = 32L * a.mp; }
        T *o = out + (size_t)slot * sstride;
        const bool vf = virt && a.vfold;   // hand-off below: agent-scope (L2-bypassing) stores
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int gg = 0; gg < 4; ++gg) {
                    const int r = Mf<T>::crow(q, gg);
                    size_t idx;
                    bool ok;
                    if (YP) { const int t = 16 * i + r, m = mb + 16 * j + l15; idx = (size_t)t * mp + m; ok = m < M; }
                    else    { const int m = mb + 16 * i + r, t = 16 * j + l15; idx = (size_t)m * 32 + t; ok = m < M; }
                    if (ok) {
                        if (vf) __hip_atomic_store(o + idx, acc[i][j][gg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        else    o[idx] = acc[i][j][gg];
                    }
                }
        if (vf && a.va + a.vb > 0) {
            // the virtual tile's contributors are workgroups 0 .. cnt0 - 1 (slots
            // 0 .. cnt0 - 1); the last to arrive sums them in slot order into
            // vout (what k_vsum did, without its launch on the chain) -- only
            // the entries the consumer reads (k in [0, va) and [128, 128 + vb))
            __shared__ int vlast;
            const int cnt0 = (a.ns - 1) / a.wst + 1;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {   // release / acquire as in brd_blk_prep.hip's Gram fold
#if BRD_HANDOFF_RELAXED
                const int old = __hip_atomic_fetch_add(a.counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
                const int old = __hip_atomic_fetch_add(a.counter, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
#endif
                const int last = old == cnt0 - 1;
                if (last) {
#if !BRD_HANDOFF_RELAXED
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#endif
                    __hip_atomic_store(a.counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                vlast = last;
            }
            __syncthreads();
            if (vlast) {
                const T *vp = (const T *)a.vpart;
                T *vo = (T *)a.vout;
                const int nk = a.va + a.vb, nel = 32 * nk;
                // entry v -> its index in the [32][256] (Y) / [256][32] (X) result
                auto at = [&](int v) {
                    if (YP) { const int t = v / nk, kk = v - t * nk; return t * kMT + (kk < a.va ? kk : 128 + kk - a.va); }
                    else    { const int kk = v >> 5, t = v & 31; return (kk < a.va ? kk : 128 + kk - a.va) * 32 + t; }
                };
#pragma unroll 1
                for (int v0 = 0; v0 < nel; v0 += 8 * kRT) {   // 8 entries a thread per round
                    T sum[8];
                    int ix[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) { sum[u] = (T)0; const int v = v0 + u * kRT + tid; ix[u] = v < nel ? at(v) : -1; }
#pragma unroll 1
                    for (int z0 = 0; z0 < cnt0; z0 += 8) {
                        T w[8][8];
#pragma unroll
                        for (int z = 0; z < 8; ++z)
#pragma unroll
                            for (int u = 0; u < 8; ++u)
                                w[z][u] = (z0 + z < cnt0 && ix[u] >= 0)
                                              ? __hip_atomic_load(vp + (size_t)(z0 + z) * 32 * kMT + ix[u], __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_AGENT)
                                              : (T)0;
#pragma unroll
                        for (int z = 0; z < 8; ++z)
#pragma unroll
                            for (int u = 0; u < 8; ++u)
                                if (z0 + z < cnt0) sum[u] += w[z][u];
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        if (ix[u] >= 0) vo[ix[u]] = sum[u];
                }
            }
        }
        if (segend == (tt + 1) * a.ns && !vf) {   // the tile's last contributor: the unused slots read 0
            for (int z = slot + 1; z < a.ksplit; ++z) {
                T *oz = out + (size_t)z * sstride;
                for (int e = tid; e < 32 * kMT; e += kRT) {
                    if (YP) { const int t = e >> 8, m = e & (kMT - 1); if (m < M) oz[(size_t)t * mp + m] = (T)0; }
                    else    { const int m = e >> 5, t = e & 31; if (m < M) oz[(size_t)m * 32 + t] = (T)0; }
                }
            }
        }
        u = segend;
        __syncthreads();   // every wave done with the ring before the next segment's DMAs
    }
}

static bool rpass_dma_enabled() {   // read per launch: parity tests switch it between calls
    const char *e = getenv("BRD_RPASS_DMA");   // A/B: 0 = the register-streaming k_rpass
    return !e || atoi(e) != 0;
}

bool rpass_dma_ok(bool yp, int K, int M, size_t elem, const void *src, long ld, const void *vsrc, long vld,
                  const void *bsrc, long bld) {
    // 16-byte vectors: no vector may straddle a source's end (Y tiles M wide,
    // X rows K long) and every row must start 16-byte aligned
    const long epv = 16 / (long)elem;
    auto al = [&](const void *p, long l) { return p == nullptr || ((uintptr_t)p % 16 == 0 && l % epv == 0); };
    return rpass_dma_enabled() && (yp ? M % epv == 0 : K % epv == 0) && al(src, ld) && al(vsrc, vld) && al(bsrc, bld);
}
int rpass_stage_k(size_t elem) { return 128 / (int)elem; }

template <typename T>
void launch_k_rpass(bool yp, dim3 grid, const RpArgs &a, const FinArgs &f, hipStream_t s, double fl, double by) {
    if (a.wst > 0) {   // the host laid the split out for k_rpass_d (rpass_dma_ok)
        if (yp) blk_launch("s1_rpass", fl, by, k_rpass_d<T, true>, grid, dim3(kRT), s, a, f);
        else    blk_launch("s1_rpass", fl, by, k_rpass_d<T, false>, grid, dim3(kRT), s, a, f);
        return;
    }
    if (yp) blk_launch("s1_rpass", fl, by, k_rpass<T, true, FinArgs>, grid, dim3(kRT), s, a, f);
    else    blk_launch("s1_rpass", fl, by, k_rpass<T, false, FinArgs>, grid, dim3(kRT), s, a, f);
}
template <typename T>
void launch_k_vsum(const T *vpart, T *vout, int nvirt, T *pbase, long pstride, const double *sgn, hipStream_t s) {
    blk_launch("s1_prep", 0.0, 0.0, k_vsum<T>, dim3(32 * kMT / 256), dim3(256), s, vpart, vout, nvirt, pbase, pstride,
               sgn);
}
template void launch_k_rpass<double>(bool, dim3, const RpArgs &, const FinArgs &, hipStream_t, double, double);
template void launch_k_rpass<float>(bool, dim3, const RpArgs &, const FinArgs &, hipStream_t, double, double);
template void launch_k_vsum<double>(const double *, double *, int, double *, long, const double *, hipStream_t);
template void launch_k_vsum<float>(const float *, float *, int, float *, long, const double *, hipStream_t);

}  // namespace blk
}  // namespace brd
