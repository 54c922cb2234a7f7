// Speculative sample groups: the start-state guess and the fold kernels.
// Part of the trace kernel's single translation unit: included by pt_kernels.hip inside its anonymous
// namespace, in this order: pt_dev_scene.h, pt_dev_walk.h, pt_dev_path.h, pt_dev_groups.h,
// pt_dev_fold.h; not a standalone header.
#pragma once

// ---- speculative sample groups: start states and the fold ---------------------
// Both run one lane per pixel, indexed like the trace kernel's items (tile, lane), so the per-item
// buffers ([item][..][64]) are read and written in whole 256-B rows.
PT_DEV bool ssg_pixel(const TraceParams& P, size_t gid, uint32_t& pos, uint32_t& lane, size_t& li)
{
    pos = (uint32_t)(gid >> 6);                      // position in the order: the per-item buffers' index
    lane = (uint32_t)(gid & 63u);
    if (pos >= P.ssgTiles) return false;
    const uint32_t tile = P.order[pos];              // packed tile coordinates
    const uint32_t tileX = tile & 0xffffu, tileY = tile >> 16;
    const uint32_t px = tileX * 8u + (lane & 7u), ly = tileY * 8u + (lane >> 3);
    li = (size_t)ly * P.width + px;
    return tileY < P.tilesY && px < P.width && ly < P.rows;
}

// Group g >= 1 of a pixel starts at draw pair round(g * n * m), m = the pixel's draw pairs per
// sample (the previous launch's, or the cost pre-pass's), strictly increasing in g; its state is
// the pixel's current state advanced that far.
__global__ void __launch_bounds__(256) ssg_guess_kernel(TraceParams P, const float* __restrict__ pairs, uint32_t n,
                                                        uint32_t* __restrict__ start)
{
    uint32_t tile, lane;
    size_t li;
    if (!ssg_pixel(P, (size_t)blockIdx.x * 256 + threadIdx.x, tile, lane, li)) return;
    const size_t npix = (size_t)P.rows * P.width;
    Xorwow st = {P.rng[li], P.rng[npix + li], P.rng[2 * npix + li], P.rng[3 * npix + li], P.rng[4 * npix + li],
                 P.rng[5 * npix + li]};
    const size_t npixAll = (size_t)P.rows * P.width;
    float m = pairs ? pairs[li] : 2.0f;
    m = (m >= 1.0f) ? fminf(m, 6.0f) : 1.0f;       // 1..6 pairs per sample (jitter + up to 5 hits)
    const float podd = pairs ? pairs[npixAll + li] : -1.0f;   // fraction of odd-length samples (< 0: unknown)
    const float var = (pairs && podd >= 0.0f) ? pairs[2 * npixAll + li] : 1.0f;   // variance of pairs per sample
    // the last group stops once its parse passes the expected end of the pixel's chain plus three
    // standard deviations (a short tail is finished by a patch round)
    const float total = (float)(P.spp * P.chunks);
    const uint32_t stopOff = (uint32_t)(total * m + 3.0f * sqrtf(total * fmaxf(var, 0.05f)) + 2.0f);
    // A pixel whose samples rarely take an odd number of pairs (< 6 %; ground under open sky: 2, or
    // 2 and 4) keeps its true sample starts on one parity for long stretches; a rare odd sample
    // flips it.  Its guesses sit on even offsets, and a second item starts one pair later, so the
    // parse that joins exists whatever the parity of the true one.  Other near-integer means q >= 3
    // use their own lattice (single item).
    const bool parityStable = podd >= 0.0f ? podd < 0.06f : fabsf(m - 2.0f) < 0.25f;
    const float q = parityStable ? 2.0f : rintf(m);
    const bool lattice = parityStable || (q >= 3.0f && fabsf(m - q) < 0.02f);
    const bool dual = parityStable && m > 1.5f;
    const uint32_t J = 2 * P.ssgG - 1;
    uint32_t off = 0;
    for (uint32_t g = 1; g < P.ssgG; ++g) {
        uint32_t o = lattice ? (uint32_t)q * (uint32_t)((float)(g * n) * (m / q) + 0.5f)
                             : (uint32_t)((float)(g * n) * m + 0.5f);
        if (o <= off) o = off + 1;
        xorwow_skip(st, 2u * (o - off));
        off = o;
        uint32_t* w = start + ((size_t)tile * J + 2 * g - 1) * kStartWords * 64 + lane;
        w[0] = o;
        w[64] = st.d;
        w[128] = st.v0;
        w[192] = st.v1;
        w[256] = st.v2;
        w[320] = st.v3;
        w[384] = st.v4;
        w[448] = g + 1 == P.ssgG ? stopOff : 0xffffffffu;
        uint32_t* w2 = w + kStartWords * 64;       // the item one pair later
        if (dual) {
            Xorwow s2 = st;
            xorwow_skip(s2, 2u);
            w2[0] = o + 1;
            w2[64] = s2.d;
            w2[128] = s2.v0;
            w2[192] = s2.v1;
            w2[256] = s2.v2;
            w2[320] = s2.v3;
            w2[384] = s2.v4;
            w2[448] = g + 1 == P.ssgG ? stopOff : 0xffffffffu;
        } else {
            w2[0] = 0xffffffffu;
        }
    }
}

// Walk each pixel's true parse through the logs.  Round 0 starts at group 0 (the pixel's own state);
// a later round starts in the patch log of the carrier that ran from the previous round's dead end.
// At every sample start the walk checks whether a later group's parse has a sample start there (its
// window bits) and, if that group logged samples from there, continues in its log.  Colours are summed
// per render() call and folded into the accumulation value exactly as trace.cu:186-198 does.  Where
// the logs end first (a dead end), the state is kept for the next round: the exact XORWOW state there
// (the item's start state advanced by the draws since), the partial sums, the next candidate group.
__global__ void __launch_bounds__(256) ssg_fold_kernel(TraceParams P, uint32_t round, const float* __restrict__ patchLog,
                                                       const uint16_t* __restrict__ patchEnd,
                                                       const uint32_t* __restrict__ patchCount, uint32_t patchCap,
                                                       float* __restrict__ pairs, uint32_t* __restrict__ deadCount)
{
    uint32_t tile, lane;
    size_t li;
    if (!ssg_pixel(P, (size_t)blockIdx.x * 256 + threadIdx.x, tile, lane, li)) return;
    const size_t npix = (size_t)P.rows * P.width;
    uint32_t* F = P.fold;
    const uint32_t G = P.ssgG, item0 = tile * (2 * G - 1), total = P.spp * P.chunks;
    f3 acc, color;
    uint32_t sIdx, c, done, off, h, odd = 0, prevRel = 0, sq = 0;
    bool inPatch;
    uint32_t cur, k, base, cnt;
    if (round == 0) {
        acc = splat(0.0f);
        if (!P.ignoreFirst) {
            const float4 a = P.accum[li];
            acc = mk(a.x, a.y, a.z);
        }
        color = splat(0.0f);
        sIdx = c = done = off = 0;
        h = 1;
        inPatch = false;
        cur = 0;
        k = 0;
        base = 0;
        cnt = P.ssgCount[(size_t)item0 * 64 + lane];
    } else {
        if (!(F[F_FLAG * npix + li] & 1u)) return;
        acc = mk(__uint_as_float(F[(F_ACC + 0) * npix + li]), __uint_as_float(F[(F_ACC + 1) * npix + li]),
                 __uint_as_float(F[(F_ACC + 2) * npix + li]));
        color = mk(__uint_as_float(F[(F_COL + 0) * npix + li]), __uint_as_float(F[(F_COL + 1) * npix + li]),
                   __uint_as_float(F[(F_COL + 2) * npix + li]));
        const uint32_t sc = F[F_SC * npix + li];
        sIdx = sc & 0xffffu;
        c = sc >> 16;
        done = F[F_DONE * npix + li];
        off = F[F_OFF * npix + li];
        h = min(F[F_H * npix + li], G);
        odd = F[F_ODD * npix + li];
        sq = F[F_SQ * npix + li];
        inPatch = true;
        cur = G;
        k = 0;
        base = off;
        cnt = patchCount[(size_t)tile * 64 + lane];
    }
    uint32_t hStart = h < G ? ssg_start_word(P, item0 + 2 * h - 1, 0, lane) : 0xffffffffu;
    while (done < total) {
        while (h < G && off > hStart + (P.ssgWin * 64u)) {
            ++h;
            hStart = h < G ? ssg_start_word(P, item0 + 2 * h - 1, 0, lane) : 0xffffffffu;
        }
        while (h + 1 < G) {                                  // the latest group started (ssg_finish)
            const uint32_t nx = ssg_start_word(P, item0 + 2 * h + 1, 0, lane);
            if (off < nx) break;
            ++h;
            hStart = nx;
        }
        if (h < G && off >= hStart) {
            bool joined = false;
            for (uint32_t ph = 0; ph < 2 && !joined; ++ph) {        // both phases of group h
                const uint32_t it = item0 + 2 * h - 1 + ph;
                if (off < hStart + ph) continue;
                const uint32_t w = off - hStart - ph;
                if (w >= (P.ssgWin * 64u)) continue;
                const unsigned long long* bits = P.ssgBits + (size_t)it * P.ssgWin * 64 + lane;
                if (!((bits[(w / 64) * 64] >> (w % 64)) & 1ull)) continue;
                uint32_t kh = __popcll(bits[(w / 64) * 64] & ((1ull << (w % 64)) - 1ull));
                for (uint32_t j = 0; j < w / 64; ++j) kh += __popcll(bits[j * 64]);
                const uint32_t ch = P.ssgCount[(size_t)it * 64 + lane];
                if (kh < ch) {                                // continue in this item's log
                    inPatch = false;
                    cur = 2 * h - 1 + ph;
                    k = kh;
                    base = hStart + ph;
                    cnt = ch;
                    joined = true;
                    prevRel = kh ? P.ssgEnd[((size_t)it * P.ssgCap + kh - 1) * 64 + lane] : 0u;
                }
            }
            if (joined) {
                ++h;
                hStart = h < G ? ssg_start_word(P, item0 + 2 * h - 1, 0, lane) : 0xffffffffu;
                continue;
            }
        }
        if (k >= cnt && !inPatch && cur >= 2 && !(cur & 1u)) {
            // a second-phase item ends where it joined its first phase: continue in that one's log
            const uint32_t it = item0 + cur - 1;
            const uint32_t w = off - (base - 1);
            const unsigned long long* bits = P.ssgBits + (size_t)it * P.ssgWin * 64 + lane;
            if (w < (P.ssgWin * 64u) && ((bits[(w / 64) * 64] >> (w % 64)) & 1ull)) {
                uint32_t kh = __popcll(bits[(w / 64) * 64] & ((1ull << (w % 64)) - 1ull));
                for (uint32_t q = 0; q < w / 64; ++q) kh += __popcll(bits[q * 64]);
                const uint32_t ch = P.ssgCount[(size_t)it * 64 + lane];
                if (kh < ch) {
                    cur -= 1;
                    k = kh;
                    base -= 1;
                    cnt = ch;
                    prevRel = kh ? P.ssgEnd[((size_t)it * P.ssgCap + kh - 1) * 64 + lane] : 0u;
                    continue;
                }
            }
        }
        if (k >= cnt) break;
        // up to 16 samples at once (their loads issued together, the sums in order); the batch ends
        // at the first sample start inside it that may be a junction or that passes group h's window,
        // which the top of the loop then handles
        uint32_t m = min(min(cnt - k, total - done), kFoldBatch);
        const float* lg = inPatch ? patchLog : P.ssgLog;
        const uint16_t* le = inPatch ? patchEnd : P.ssgEnd;
        const size_t rec = inPatch ? (size_t)tile * patchCap + k : (size_t)(item0 + cur) * P.ssgCap + k;
        float cx[kFoldBatch], cy[kFoldBatch], cz[kFoldBatch];
        uint32_t er[kFoldBatch];
#pragma unroll
        for (uint32_t j = 0; j < kFoldBatch; ++j) {
            if (j < m) {
                cx[j] = lg[((rec + j) * 3 + 0) * 64 + lane];
                cy[j] = lg[((rec + j) * 3 + 1) * 64 + lane];
                cz[j] = lg[((rec + j) * 3 + 2) * 64 + lane];
                er[j] = le[(rec + j) * 64 + lane];
            }
        }
        if (h < G && m > 1 && base + er[m - 2] >= hStart) {
            // bit words of both phases around the batch's first start at or past hStart
            const uint32_t p0 = max(base + er[0], hStart) - hStart;
            const uint32_t i0 = min(p0 / 64, P.ssgWin - 1);
            const unsigned long long* bA = P.ssgBits + (size_t)(item0 + 2 * h - 1) * P.ssgWin * 64 + lane;
            const unsigned long long* bB = bA + (size_t)P.ssgWin * 64;
            const unsigned long long a0 = bA[i0 * 64], a1 = i0 + 1 < P.ssgWin ? bA[(i0 + 1) * 64] : 0ull;
            const uint32_t iB = p0 ? min((p0 - 1) / 64, P.ssgWin - 1) : 0u;
            const unsigned long long c0 = bB[iB * 64], c1 = iB + 1 < P.ssgWin ? bB[(iB + 1) * 64] : 0ull;
            auto bit = [&](unsigned long long w0, unsigned long long w1, uint32_t i, const unsigned long long* b,
                           uint32_t w) -> bool {
                const uint32_t idx = w / 64;
                const unsigned long long word = idx == i ? w0 : (idx == i + 1 ? w1 : (idx < P.ssgWin ? b[idx * 64] : 0ull));
                return (word >> (w % 64)) & 1ull;
            };
            const uint32_t hNext = h + 1 < G ? ssg_start_word(P, item0 + 2 * h + 1, 0, lane) : 0xffffffffu;
            for (uint32_t j = 0; j + 1 < m; ++j) {
                const uint32_t pos = base + er[j];
                if (pos < hStart) continue;
                const uint32_t w = pos - hStart;
                if (w > (P.ssgWin * 64u) || pos >= hNext || (w < (P.ssgWin * 64u) && bit(a0, a1, i0, bA, w)) ||
                    (w >= 1 && bit(c0, c1, iB, bB, w - 1))) {
                    m = j + 1;
                    break;
                }
            }
        }
        uint32_t endRel = prevRel;
#pragma unroll
        for (uint32_t j = 0; j < kFoldBatch; ++j) {
            if (j < m) {
                odd += (er[j] - endRel) & 1u;               // odd-length sample (guess statistics)
                sq += (er[j] - endRel) * (er[j] - endRel);
                endRel = er[j];
            }
        }
        prevRel = endRel;
#pragma unroll
        for (uint32_t j = 0; j < kFoldBatch; ++j) {
            if (j < m) {
                color = add(color, mk(cx[j], cy[j], cz[j]));
                if (++sIdx == P.spp) {                                  // trace.cu:196
                    acc = (c == 0 && P.ignoreFirst) ? color : add(color, acc);
                    color = splat(0.0f);
                    sIdx = 0;
                    ++c;
                }
            }
        }
        off = base + endRel;
        k += m;
        done += m;
    }
    // the exact state at `off`: the current item's start state advanced by the draws since
    Xorwow st;
    if (inPatch) {
        st = {F[(F_ST + 0) * npix + li], F[(F_ST + 1) * npix + li], F[(F_ST + 2) * npix + li],
              F[(F_ST + 3) * npix + li], F[(F_ST + 4) * npix + li], F[(F_ST + 5) * npix + li]};
    } else if (cur == 0) {
        st = {P.rng[li], P.rng[npix + li], P.rng[2 * npix + li], P.rng[3 * npix + li], P.rng[4 * npix + li],
              P.rng[5 * npix + li]};
    } else {
        const uint32_t it = item0 + cur;
        st = {ssg_start_word(P, it, 1, lane), ssg_start_word(P, it, 2, lane), ssg_start_word(P, it, 3, lane),
              ssg_start_word(P, it, 4, lane), ssg_start_word(P, it, 5, lane), ssg_start_word(P, it, 6, lane)};
    }
    xorwow_skip(st, 2u * (off - base));
    P.rng[li] = st.d;
    P.rng[npix + li] = st.v0;
    P.rng[2 * npix + li] = st.v1;
    P.rng[3 * npix + li] = st.v2;
    P.rng[4 * npix + li] = st.v3;
    P.rng[5 * npix + li] = st.v4;
    P.accum[li] = make_float4(acc.x, acc.y, acc.z, 1.0f);
    if (done == total) {
        if (done > 0) {
            pairs[li] = (float)off / (float)done;
            pairs[npix + li] = (float)odd / (float)done;
            const float mean = (float)off / (float)done;
            pairs[2 * npix + li] = fmaxf((float)sq / (float)done - mean * mean, 0.0f);
        }
        F[F_FLAG * npix + li] = round << 8;      // finished (bit 0 clear), in this fold round (diagnostics)
        return;
    }
    if (done > 0) pairs[li] = (float)off / (float)done;   // the next launch's guess for this pixel
    F[(F_ACC + 0) * npix + li] = __float_as_uint(acc.x);
    F[(F_ACC + 1) * npix + li] = __float_as_uint(acc.y);
    F[(F_ACC + 2) * npix + li] = __float_as_uint(acc.z);
    F[(F_COL + 0) * npix + li] = __float_as_uint(color.x);
    F[(F_COL + 1) * npix + li] = __float_as_uint(color.y);
    F[(F_COL + 2) * npix + li] = __float_as_uint(color.z);
    F[F_SC * npix + li] = sIdx | (c << 16);
    F[F_DONE * npix + li] = done;
    F[F_OFF * npix + li] = off;
    F[F_H * npix + li] = h;
    F[F_ODD * npix + li] = odd;
    F[F_SQ * npix + li] = sq;
    F[(F_ST + 0) * npix + li] = st.d;
    F[(F_ST + 1) * npix + li] = st.v0;
    F[(F_ST + 2) * npix + li] = st.v1;
    F[(F_ST + 3) * npix + li] = st.v2;
    F[(F_ST + 4) * npix + li] = st.v3;
    F[(F_ST + 5) * npix + li] = st.v4;
    F[F_FLAG * npix + li] = 1u;
    atomicAdd(deadCount, 1u);
}
