// pull_kernel.h -- k_pull, the CSR pull over the bit-sliced frontier (included by engine.hip,
// which defines WordCtl, PullArgs and group_fix).
//
// One tick of P2PNode::HandleRead -> processedShares check -> ReceiveShare ->
// GossipShareToPeers (p2pnode.cc:127-199) for every node at once:
//     inc = OR_{u in peers(v)} F_cur[u];  new = inc & ~seen[v] & keep;  seen |= new;
//     F_next[v] = new;  recv[v] += popcount(new);  sent[v] += |peers(v)| * popcount(new)
//
// Lane layout: a node is served by GRP = LPW x EPN lanes.  Word-lane wl owns the 16-B word pair
// [2wl, 2wl+1] of every 2*LPW-word pass; edge-lane el takes every EPN-th peer.  Wide windows
// (sparse graphs) use EPN = 1, LPW = 64: a wave reads 1 KiB of one peer row per instruction.
// Narrow windows on dense graphs use EPN > 1: lanes split the peer list, then OR-reduce.
// A launch covers the words [wbase, wbase + wact) of every row (wact <= kPullLdsWords).
//
// Per-word state shared by all nodes (last tick's liveness, the word flags) is staged in LDS
// once per block, so a work item carries only its own seen pair between pipeline stages.
//
// Latency structure.  The pull is a dependent-load chain per node (row_ptr -> peer ids ->
// peer occupancy words -> peer rows), so the kernel pipelines it: a wave owns 64 consecutive
// nodes and loads their row_ptr once; work items (node, pass) run in order, and in iteration k
// the kernel issues the own seen pair of item k+1, the peer ids of item k+2 and the peer
// occupancy words of item k+1 before the peer-row gathers of item k, so one round trip per
// item covers the whole chain.  Peer rows are gathered kInflight at a time (16 B per lane each).
//
// Work skipping (bytes the pull never moves):
//   dead pair  -- no column of the two words had a frontier bit anywhere last tick
//                 (live_prev == 0): nothing can arrive;
//   saturated  -- the node has seen every live column of the pair: peer rows not read;
//   empty row  -- a peer's 16-word tile row with no frontier bit (its occupancy bit in
//                 nz_cur is clear) is not read: young tiles are mostly empty rows;
//   F_next tile rows are written only when some word of the tile got a bit (and the tile's
//   occupancy bit set); rows left unwritten hold stale bits that no reader ever loads.
#pragma once

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long x) {
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

// Lanes of the wave for which c holds (a wave-uniform value: traffic accounting in SGPRs).
__device__ __forceinline__ uint32_t wave_count(bool c) { return (uint32_t)__popcll(__ballot(c)); }

enum : uint32_t { WF_CLEAR = 1u, WF_GROUP = 2u, WF_KEEP = 4u, WF_SNAP = 8u };

constexpr uint32_t kPullLdsWords = 2048;  // words per launch: LDS liveness, new liveness, flags
#ifndef PULL_INFLIGHT
#define PULL_INFLIGHT 8
#endif
constexpr int kInflight = PULL_INFLIGHT;  // peer-row loads in flight per lane

__host__ __device__ constexpr size_t pull_lds_bytes(uint32_t wact) {
    return (size_t)wact * 16u + (((size_t)wact + 15u) & ~(size_t)15u);
}

// Peer ids of the first GRP peers of item k's node (0xffffffff past the list).
template <int LPW, int EPN>
__device__ __forceinline__ uint32_t pull_cid_load(const PullArgs& a, uint32_t step, uint64_t c0,
                                                  int64_t rp, int64_t rp_end, uint32_t gl,
                                                  uint32_t slot) {
    constexpr int NPW = 64 / (LPW * EPN);
    const uint32_t idx = step * NPW + slot;
    const int32_t beg = __shfl((int)rp, (int)idx, 64);
    const int32_t nx = __shfl((int)rp, (int)((idx + 1u) & 63u), 64);
    const int32_t end = (idx + 1u < 64u) ? nx : (int32_t)rp_end;
    const int32_t jj = beg + (int32_t)gl;
    return (c0 + idx < a.n && jj < end) ? (uint32_t)a.col[jj] : 0xffffffffu;
}

template <int LPW, int EPN>
__global__ __launch_bounds__(256) void k_pull(PullArgs a) {
    constexpr int GRP = LPW * EPN;  // lanes per node
    constexpr int NPW = 64 / GRP;   // nodes per wave step
    static_assert(GRP <= 64 && (64 % GRP) == 0, "lane layout");
    extern __shared__ unsigned long long smem[];
    unsigned long long* s_lp = smem;             // live_prev of this launch's words
    unsigned long long* s_new = smem + a.wact;   // liveness of this tick (OR of new bits)
    uint8_t* s_wf = reinterpret_cast<uint8_t*>(smem + 2u * a.wact);
    for (uint32_t i = threadIdx.x; i < a.wact; i += 256) {
        s_lp[i] = (a.live_prev && !a.noskip) ? a.live_prev[a.wbase + i] : ~0ull;
        s_new[i] = 0ull;
        s_wf[i] = a.wflags[a.wbase + i];
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gl = lane % GRP, wl = gl % LPW, el = gl / LPW, slot = lane / GRP;
    const uint64_t stride = a.stride;
    const uint64_t n = a.n;
    const uint64_t wave = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * 4u;
    const uint32_t npass = (a.wact + 2u * LPW - 1u) / (2u * LPW);
    const uint32_t nsteps = 64u / NPW;
    unsigned long long snap_local = 0ull;
    uint32_t t_pe = 0, t_col = 0, t_srd = 0, t_swr = 0, t_fwr = 0, t_nz = 0;  // wave-uniform
    unsigned long long nzacc = 0ull;
    const bool gather = a.inc == nullptr && EPN == 1;  // the pipelined id/occupancy loads

    for (uint64_t c0 = wave * 64u; c0 < n; c0 += nwaves * 64u) {
        const int64_t rp = a.rowptr[min(c0 + lane, n)];
        const int64_t rp_end = a.rowptr[min(c0 + 64u, n)];
        // item k = (step, pass): node c0 + step * NPW + slot, words wbase + pass * 2 LPW + 2 wl
        uint32_t step = 0, pass = 0;
        ulonglong2 s2c = make_ulonglong2(0ull, 0ull);
        {
            const uint64_t v = c0 + slot;
            const uint32_t w = a.wbase + 2u * wl;
            if (v < n && w < a.wbase + a.wact) s2c = *reinterpret_cast<const ulonglong2*>(a.seen + v * stride + w);
        }
        uint32_t cid0 = 0xffffffffu, cid1 = 0xffffffffu;
        unsigned long long nz0 = 0ull;
        if (gather) {
            cid0 = pull_cid_load<LPW, EPN>(a, 0u, c0, rp, rp_end, gl, slot);
            cid1 = npass > 1u ? cid0 : pull_cid_load<LPW, EPN>(a, 1u, c0, rp, rp_end, gl, slot);
            nz0 = cid0 != 0xffffffffu ? a.nz_cur[(uint64_t)cid0 * a.ntw + (a.wbase >> 10)] : 0ull;
            t_nz += wave_count(cid0 != 0xffffffffu);
        }
        uint32_t cnt = 0;
        while (step < nsteps) {
            // ---- geometry of this item and the next two ----
            const uint32_t step1 = pass + 1u < npass ? step : step + 1u;
            const uint32_t pass1 = pass + 1u < npass ? pass + 1u : 0u;
            const uint32_t step2 = pass1 + 1u < npass ? step1 : step1 + 1u;
            const uint32_t idx = step * NPW + slot;
            const uint32_t v = (uint32_t)(c0 + idx);
            const uint32_t w = a.wbase + pass * 2u * LPW + 2u * wl;
            const bool act = c0 + idx < n && w < a.wbase + a.wact;
            // ---- stage loads: own seen pair of item k+1, ids of k+2, occupancy of k+1 ----
            ulonglong2 s2n = make_ulonglong2(0ull, 0ull);
            if (step1 < nsteps) {
                const uint64_t v1 = c0 + step1 * NPW + slot;
                const uint32_t w1 = a.wbase + pass1 * 2u * LPW + 2u * wl;
                if (v1 < n && w1 < a.wbase + a.wact)
                    s2n = *reinterpret_cast<const ulonglong2*>(a.seen + v1 * stride + w1);
            }
            uint32_t cid2 = 0xffffffffu;
            unsigned long long nz1 = 0ull;
            if (gather) {
                if (step2 < nsteps)
                    cid2 = step2 == step1 ? cid1 : pull_cid_load<LPW, EPN>(a, step2, c0, rp, rp_end, gl, slot);
                if (step1 < nsteps) {
                    const uint32_t tw1 = (a.wbase + pass1 * 2u * LPW) >> 10;
                    const uint32_t tw0 = (a.wbase + pass * 2u * LPW) >> 10;
                    if (step1 == step && tw1 == tw0) {
                        nz1 = nz0;  // same node, same occupancy word
                    } else {
                        nz1 = cid1 != 0xffffffffu ? a.nz_cur[(uint64_t)cid1 * a.ntw + tw1] : 0ull;
                        t_nz += wave_count(cid1 != 0xffffffffu);
                    }
                }
            }
            // ---- decide: is any peer row worth reading for this pair? ----
            uint32_t f0 = 0, f1 = 0;
            uint64_t lp0 = 0ull, lp1 = 0ull;
            if (act) {
                const uint32_t lw = w - a.wbase;
                const uint16_t fl = *reinterpret_cast<const uint16_t*>(s_wf + lw);
                f0 = fl & 0xffu;
                f1 = fl >> 8;
                lp0 = s_lp[lw];
                lp1 = s_lp[lw + 1u];
            }
            const bool dead = (lp0 | lp1) == 0ull;
            ulonglong2 s2 = s2c;
            if (f0 & WF_CLEAR) s2.x = 0ull;
            if (f1 & WF_CLEAR) s2.y = 0ull;
            uint64_t k0 = ~0ull, k1 = ~0ull;
            if (act && (f0 & WF_KEEP)) k0 = a.ctl[w].keep;
            if (act && (f1 & WF_KEEP)) k1 = a.ctl[w + 1].keep;
            // (incoming mode must consume every live pair's incoming word: no saturation skip)
            const bool need = act && !dead &&
                              (a.noskip || a.inc || ((lp0 & ~s2.x & k0) | (lp1 & ~s2.y & k1)) != 0ull);
            // Columns are allocated in 16-word tiles (one 128-B line per row, engine.hip), so the
            // read decision is made per tile: the 8 word-lanes of a tile load together and every
            // fetched line is fully used.
            int tn = need ? 1 : 0;
            tn |= __shfl_xor(tn, 1, GRP);
            tn |= __shfl_xor(tn, 2, GRP);
            tn |= __shfl_xor(tn, 4, GRP);
            const bool tneed = tn != 0 && act;
            int gneed = tn;
#pragma unroll
            for (int off = GRP / 2; off > 4; off >>= 1) gneed |= __shfl_xor(gneed, off, GRP);
            // ---- gather peer rows ----
            const uint32_t tw = w >> 10;  // one occupancy word per pass: a pass spans <= 8 tiles of 64
            const unsigned long long tbit = 1ull << ((w >> 4) & 63u);
            const int32_t beg = __shfl((int)rp, (int)idx, 64);
            const int32_t nxb = __shfl((int)rp, (int)((idx + 1u) & 63u), 64);
            const int32_t end = (idx + 1u < 64u) ? nxb : (int32_t)rp_end;
            uint64_t acc0 = 0ull, acc1 = 0ull;
            if (a.inc) {
                // DENSE mode: the gather already happened as an MFMA contraction; take the
                // incoming words and leave them zeroed for the next tick.
                if (tneed && el == 0) {
                    ulonglong2* ip = reinterpret_cast<ulonglong2*>(a.inc + (uint64_t)v * stride + w);
                    const ulonglong2 x = *ip;
                    acc0 = x.x;
                    acc1 = x.y;
                    if ((acc0 | acc1) != 0ull) *ip = make_ulonglong2(0ull, 0ull);
                }
            } else if (gneed) {  // uniform inside the node group
                const uint64_t* Fw = a.Fcur + w;
                if constexpr (EPN == 1) {
                    for (int32_t cb = beg; cb < end; cb += GRP) {
                        uint32_t cid = cid0;
                        unsigned long long nzw = nz0;
                        const int rem = min(GRP, end - cb);
                        if (cb != beg) {  // peers beyond the first GRP: loaded inline (rare)
                            const int32_t jj = cb + (int32_t)gl;
                            cid = (jj < end) ? (uint32_t)a.col[jj] : 0u;
                            nzw = ((int)gl < rem) ? a.nz_cur[(uint64_t)cid * a.ntw + tw] : 0ull;
                            t_nz += wave_count((int)gl < rem);
                        }
                        t_col += wave_count((int)gl < rem);
                        // the <= 8 occupancy bits of this pass's tiles, tested per lane by tile
                        const uint32_t nzp = (uint32_t)(nzw >> ((((w - 2u * wl) >> 4)) & 63u)) & 0xffu;
                        for (int t0 = 0; t0 < rem; t0 += kInflight) {
                            uint32_t u[kInflight], z[kInflight];
#pragma unroll
                            for (int t = 0; t < kInflight; t++) {
                                u[t] = (uint32_t)__shfl((int)cid, (t0 + t) & (GRP - 1), GRP);
                                z[t] = (uint32_t)__shfl((int)nzp, (t0 + t) & (GRP - 1), GRP);
                            }
                            ulonglong2 q[kInflight];
                            uint32_t hits = 0u;
#pragma unroll
                            for (int t = 0; t < kInflight; t++) {
                                q[t] = make_ulonglong2(0ull, 0ull);
                                const bool hit = ((z[t] >> (wl >> 3)) & 1u) != 0u;
                                hits |= hit ? (1u << t) : 0u;
                                const bool issue = tneed && t0 + t < rem && (hit || a.noskip);
                                if (issue) q[t] = *reinterpret_cast<const ulonglong2*>(Fw + (uint64_t)u[t] * stride);
                                t_pe += wave_count(issue);
                            }
                            // (consumed after all 8 loads are in flight; a row loaded without its
                            // occupancy bit -- NOSKIP diagnostic only -- is stale and dropped)
#pragma unroll
                            for (int t = 0; t < kInflight; t++) {
                                const bool h = (hits >> t) & 1u;
                                acc0 |= h ? q[t].x : 0ull;
                                acc1 |= h ? q[t].y : 0ull;
                            }
                        }
                    }
                } else {
                    // edge-lane el walks peers beg+el, beg+el+EPN, ...; 8 in flight
                    for (int32_t j0 = beg + (int32_t)el; j0 < end; j0 += 8 * EPN) {
                        uint32_t u[8];
                        unsigned long long z[8];
#pragma unroll
                        for (int t = 0; t < 8; t++) {
                            const int32_t j = j0 + t * EPN;
                            u[t] = (tneed && j < end) ? (uint32_t)a.col[j] : 0xffffffffu;
                            t_col += wave_count(wl == 0 && u[t] != 0xffffffffu);
                        }
#pragma unroll
                        for (int t = 0; t < 8; t++) {
                            z[t] = 0ull;
                            if (u[t] != 0xffffffffu) z[t] = a.nz_cur[(uint64_t)u[t] * a.ntw + tw];
                            t_nz += wave_count(u[t] != 0xffffffffu);
                        }
                        ulonglong2 q[8];
                        uint32_t hits = 0u;
#pragma unroll
                        for (int t = 0; t < 8; t++) {
                            q[t] = make_ulonglong2(0ull, 0ull);
                            const bool hit = (z[t] & tbit) != 0ull;
                            hits |= hit ? (1u << t) : 0u;
                            const bool issue = u[t] != 0xffffffffu && (hit || a.noskip);
                            if (issue) q[t] = *reinterpret_cast<const ulonglong2*>(Fw + (uint64_t)u[t] * stride);
                            t_pe += wave_count(issue);
                        }
#pragma unroll
                        for (int t = 0; t < 8; t++) {
                            const bool h = (hits >> t) & 1u;
                            acc0 |= h ? q[t].x : 0ull;
                            acc1 |= h ? q[t].y : 0ull;
                        }
                    }
                }
            }
            if constexpr (EPN > 1) {
#pragma unroll
                for (int off = LPW; off < GRP; off <<= 1) {
                    acc0 |= __shfl_xor(acc0, off, GRP);
                    acc1 |= __shfl_xor(acc1, off, GRP);
                }
            }
            // ---- dedup ----
            uint64_t n0 = 0ull, n1 = 0ull;
            if (act && el == 0 && !dead) {
                n0 = acc0 & ~s2.x & k0;
                n1 = acc1 & ~s2.y & k1;
                if (f0 & WF_GROUP) n0 = group_fix(n0, s2.x, a.ctl[w].gmask, a.ctl[w].gstart);
                if (f1 & WF_GROUP) n1 = group_fix(n1, s2.y, a.ctl[w + 1].gmask, a.ctl[w + 1].gstart);
            }
            // tile occupancy of F_next: the 8 word-lanes of a tile agree on writing the row
            int ta = (n0 | n1) != 0ull;
            ta |= __shfl_xor(ta, 1, GRP);
            ta |= __shfl_xor(ta, 2, GRP);
            ta |= __shfl_xor(ta, 4, GRP);
            // ---- state, counters (one lane per word pair) ----
            const bool own = act && el == 0;
            const bool swr = own && (dead ? ((f0 | f1) & WF_CLEAR) != 0u
                                          : ((n0 | n1) != 0ull || ((f0 | f1) & WF_CLEAR) != 0u));
            t_fwr += wave_count(own && ta);
            t_srd += wave_count(own && !dead);
            t_swr += wave_count(swr);
            if (own) {
                uint64_t* sp = a.seen + (uint64_t)v * stride + w;
                uint64_t* fp = a.Fnext + (uint64_t)v * stride + w;
                if (ta) *reinterpret_cast<ulonglong2*>(fp) = make_ulonglong2(n0, n1);
                if (swr) {
                    if (dead && !((f0 & f1) & WF_CLEAR))
                        sp[(f0 & WF_CLEAR) ? 0 : 1] = 0ull;
                    else
                        *reinterpret_cast<ulonglong2*>(sp) = make_ulonglong2(s2.x | n0, s2.y | n1);
                }
                if (!dead) {
                    cnt += (uint32_t)(__popcll(n0) + __popcll(n1));
                    if (a.snap) {
                        if (f0 & WF_SNAP) snap_local += (unsigned long long)__popcll(n0 & a.ctl[w].snap);
                        if (f1 & WF_SNAP) snap_local += (unsigned long long)__popcll(n1 & a.ctl[w + 1].snap);
                    }
                    if (n0) atomicOr(&s_new[w - a.wbase], (unsigned long long)n0);
                    if (n1) atomicOr(&s_new[w + 1 - a.wbase], (unsigned long long)n1);
                }
            }
            // ---- occupancy word of this node, written whole once per nz word index ----
            {
                unsigned long long nb = (ta && own && (wl & 7u) == 0u) ? tbit : 0ull;
#pragma unroll
                for (int off = GRP / 2; off > 0; off >>= 1) nb |= __shfl_xor(nb, off, GRP);
                nzacc |= nb;
                const bool last_of_tw = pass + 1u == npass || ((a.wbase + (pass + 1u) * 2u * LPW) >> 10) != tw;
                if (last_of_tw) {
                    if (gl == 0 && c0 + idx < n) a.nz_next[(uint64_t)v * a.ntw + tw] = nzacc;
                    nzacc = 0ull;
                }
            }
            // ---- per-node counters after the node's last pass ----
            if (pass + 1u == npass) {
                uint32_t c = cnt;
#pragma unroll
                for (int off = GRP / 2; off > 0; off >>= 1) c += __shfl_xor(c, off, GRP);
                if (gl == 0 && c) {
                    a.recv[v] += c;
                    a.sent[v] += (uint64_t)c * a.deg[v];
                }
                cnt = 0;
            }
            // ---- advance the pipeline ----
            s2c = s2n;
            cid0 = cid1;
            cid1 = cid2;
            nz0 = nz1;
            step = step1;
            pass = pass1;
        }
    }
    if (a.snap) {
        snap_local = wave_sum(snap_local);
        if (lane == 0 && snap_local) atomicAdd(a.snap, snap_local);
    }
    if (a.acct && lane == 0) {
        const uint32_t tv[6] = {t_pe, t_col, t_srd, t_swr, t_fwr, t_nz};
        const int slot_of[6] = {0, 1, 2, 3, 4, 7};
#pragma unroll
        for (int q = 0; q < 6; q++)
            if (tv[q]) atomicAdd(&a.acct[slot_of[q]], (unsigned long long)tv[q]);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < a.wact; i += 256) {
        const unsigned long long x = s_new[i];
        if (x) atomicOr(&a.live[a.wbase + i], x);
    }
}
