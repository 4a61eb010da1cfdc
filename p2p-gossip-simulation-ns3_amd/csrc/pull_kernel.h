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
//
// Latency structure.  The pull is a dependent-load chain per node (row_ptr -> peer ids / own
// seen row -> peer rows), so the kernel pipelines it: a wave owns 64 consecutive nodes and
// loads their row_ptr once; work items (node, pass) are processed in order and the per-item
// "stage A" loads (word flags, last two ticks' liveness, own seen pair, first 64 peer ids) of
// item k+1 are issued before the peer-row gathers of item k, so they ride in the same round
// trip.  Peer rows are gathered 8 at a time (8 x 16 B per lane in flight).
//
// Work skipping (bytes the pull never moves):
//   dead pair  -- no column of the two words had a frontier bit anywhere last tick
//                 (live_prev == 0): nothing can arrive;
//   saturated  -- the node has seen every live column of the pair: peer rows not read;
//   F_next is written only where the overwritten buffer (tick t-2) may hold bits.
#pragma once

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long x) {
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

enum : uint32_t { WF_CLEAR = 1u, WF_GROUP = 2u, WF_KEEP = 4u, WF_SNAP = 8u };

struct PullStage {
    uint32_t v;
    int32_t beg, end;  // nnz < 2^31 (checked in gossip_engine_set_graph)
    uint32_t w, pass;
    uint32_t f0, f1;
    uint64_t lp0, lp1;
    ulonglong2 s2;
    uint32_t cid;
    bool act, pp_dirty;
};

template <int LPW, int EPN>
__device__ __forceinline__ void pull_stage_load(const PullArgs& a, PullStage& st, uint32_t k,
                                                uint32_t npass, uint64_t c0, int64_t rp,
                                                int64_t rp_end, uint32_t gl, uint32_t wl,
                                                uint32_t slot) {
    constexpr int GRP = LPW * EPN;
    constexpr int NPW = 64 / GRP;
    const uint32_t step = k / npass, p = k - step * npass;
    const uint32_t idx = step * NPW + slot;
    st.v = (uint32_t)(c0 + idx);
    st.beg = __shfl((int)rp, (int)idx, 64);
    const int32_t nx = __shfl((int)rp, (int)((idx + 1u) & 63u), 64);
    st.end = (idx + 1u < 64u) ? nx : (int32_t)rp_end;
    st.pass = p;
    st.w = p * 2u * LPW + 2u * wl;
    st.act = c0 + idx < a.n && st.w < a.wact;
    st.f0 = st.f1 = 0;
    st.lp0 = st.lp1 = 0ull;
    st.pp_dirty = false;
    st.s2 = make_ulonglong2(0ull, 0ull);
    st.cid = 0u;
    if (st.act) {
        const uint16_t fl = *reinterpret_cast<const uint16_t*>(a.wflags + st.w);
        st.f0 = fl & 0xffu;
        st.f1 = fl >> 8;
        st.lp0 = (a.live_prev && !a.noskip) ? a.live_prev[st.w] : ~0ull;
        st.lp1 = (a.live_prev && !a.noskip) ? a.live_prev[st.w + 1] : ~0ull;
        st.pp_dirty = a.live_pp ? ((a.live_pp[st.w] | a.live_pp[st.w + 1]) != 0ull) : true;
        st.s2 = *reinterpret_cast<const ulonglong2*>(a.seen + (uint64_t)st.v * a.stride + st.w);
    }
    if constexpr (EPN == 1) {
        const int32_t jj = st.beg + (int32_t)gl;
        if (c0 + idx < a.n && jj < st.end) st.cid = (uint32_t)a.col[jj];
    }
}

template <int LPW, int EPN>
__global__ __launch_bounds__(256) void k_pull(PullArgs a) {
    constexpr int GRP = LPW * EPN;  // lanes per node
    constexpr int NPW = 64 / GRP;   // nodes per wave step
    static_assert(GRP <= 64 && (64 % GRP) == 0, "lane layout");
    extern __shared__ unsigned long long s_live[];
    if (a.use_lds) {
        for (uint32_t i = threadIdx.x; i < a.wact; i += 256) s_live[i] = 0ull;
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gl = lane % GRP, wl = gl % LPW, el = gl / LPW, slot = lane / GRP;
    const uint64_t stride = a.stride;
    const uint64_t n = a.n;
    const uint64_t wave = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * 4u;
    const uint32_t npass = (a.wact + 2u * LPW - 1u) / (2u * LPW);
    const uint32_t nitems = (64u / NPW) * npass;
    unsigned long long snap_local = 0ull;
    unsigned long long t_pe = 0, t_col = 0, t_srd = 0, t_swr = 0, t_fwr = 0;

    for (uint64_t c0 = wave * 64u; c0 < n; c0 += nwaves * 64u) {
        const int64_t rp = a.rowptr[min(c0 + lane, n)];
        const int64_t rp_end = a.rowptr[min(c0 + 64u, n)];
        PullStage cur, nxt;
        pull_stage_load<LPW, EPN>(a, cur, 0u, npass, c0, rp, rp_end, gl, wl, slot);
        uint32_t cnt = 0;
        for (uint32_t k = 0; k < nitems; k++) {
            if (k + 1u < nitems) pull_stage_load<LPW, EPN>(a, nxt, k + 1u, npass, c0, rp, rp_end, gl, wl, slot);
            // ---- decide: is any peer row worth reading for this pair? ----
            const bool dead = (cur.lp0 | cur.lp1) == 0ull;
            ulonglong2 s2 = cur.s2;
            if (cur.f0 & WF_CLEAR) s2.x = 0ull;
            if (cur.f1 & WF_CLEAR) s2.y = 0ull;
            uint64_t k0 = ~0ull, k1 = ~0ull;
            if (cur.act && (cur.f0 & WF_KEEP)) k0 = a.ctl[cur.w].keep;
            if (cur.act && (cur.f1 & WF_KEEP)) k1 = a.ctl[cur.w + 1].keep;
            // (incoming mode must consume every live pair's incoming word: no saturation skip)
            const bool need = cur.act && !dead &&
                              (a.noskip || a.inc || ((cur.lp0 & ~s2.x & k0) | (cur.lp1 & ~s2.y & k1)) != 0ull);
            // Columns are allocated in 16-word tiles (one 128-B line per row, engine.hip), so the
            // read decision is made per tile: the 8 word-lanes of a tile load together and every
            // fetched line is fully used.
            int tn = need ? 1 : 0;
            tn |= __shfl_xor(tn, 1, GRP);
            tn |= __shfl_xor(tn, 2, GRP);
            tn |= __shfl_xor(tn, 4, GRP);
            const bool tneed = tn != 0 && cur.act;
            int gneed = tn;
#pragma unroll
            for (int off = GRP / 2; off > 4; off >>= 1) gneed |= __shfl_xor(gneed, off, GRP);
            // ---- gather peer rows ----
            uint64_t acc0 = 0ull, acc1 = 0ull;
            if (a.inc) {
                // DENSE mode: the gather already happened as an MFMA contraction; take the
                // incoming words and leave them zeroed for the next tick.
                if (tneed && el == 0) {
                    ulonglong2* ip = reinterpret_cast<ulonglong2*>(a.inc + (uint64_t)cur.v * stride + cur.w);
                    const ulonglong2 x = *ip;
                    acc0 = x.x;
                    acc1 = x.y;
                    if ((acc0 | acc1) != 0ull) *ip = make_ulonglong2(0ull, 0ull);
                }
            } else if (gneed) {  // uniform inside the node group
                const uint64_t* Fw = a.Fcur + cur.w;
                const int32_t beg = cur.beg, end = cur.end;
                if constexpr (EPN == 1) {
                    for (int32_t cb = beg; cb < end; cb += GRP) {
                        uint32_t cid = cur.cid;
                        if (cb != beg) {
                            const int32_t jj = cb + (int32_t)gl;
                            cid = (jj < end) ? (uint32_t)a.col[jj] : 0u;
                        }
                        const int rem = min(GRP, end - cb);
                        for (int t0 = 0; t0 < rem; t0 += 8) {
                            uint32_t u[8];
#pragma unroll
                            for (int t = 0; t < 8; t++) u[t] = (uint32_t)__shfl((int)cid, (t0 + t) & (GRP - 1), GRP);
                            ulonglong2 q[8];
#pragma unroll
                            for (int t = 0; t < 8; t++) {
                                q[t] = make_ulonglong2(0ull, 0ull);
                                if (tneed && t0 + t < rem)
                                    q[t] = *reinterpret_cast<const ulonglong2*>(Fw + (uint64_t)u[t] * stride);
                            }
#pragma unroll
                            for (int t = 0; t < 8; t++) {
                                acc0 |= q[t].x;
                                acc1 |= q[t].y;
                            }
                        }
                        if (gl == 0) t_col += (unsigned long long)rem;  // one coalesced id load per group
                    }
                    if (tneed) t_pe += (unsigned long long)(end - beg);
                } else {
                    // edge-lane el walks peers beg+el, beg+el+EPN, ...; 8 in flight
                    for (int32_t j0 = beg + (int32_t)el; j0 < end; j0 += 8 * EPN) {
                        uint32_t u[8];
#pragma unroll
                        for (int t = 0; t < 8; t++) {
                            const int32_t j = j0 + t * EPN;
                            u[t] = (tneed && j < end) ? (uint32_t)a.col[j] : 0xffffffffu;
                        }
                        ulonglong2 q[8];
#pragma unroll
                        for (int t = 0; t < 8; t++) {
                            q[t] = make_ulonglong2(0ull, 0ull);
                            if (u[t] != 0xffffffffu)
                                q[t] = *reinterpret_cast<const ulonglong2*>(Fw + (uint64_t)u[t] * stride);
                        }
#pragma unroll
                        for (int t = 0; t < 8; t++) {
                            acc0 |= q[t].x;
                            acc1 |= q[t].y;
                            t_col += (wl == 0 && u[t] != 0xffffffffu) ? 1u : 0u;
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
                if (tneed && el == 0) t_pe += (unsigned long long)(cur.end - cur.beg);
            }
            // ---- dedup, state, counters (one lane per word pair) ----
            if (cur.act && el == 0) {
                uint64_t* sp = a.seen + (uint64_t)cur.v * stride + cur.w;
                uint64_t* fp = a.Fnext + (uint64_t)cur.v * stride + cur.w;
                if (dead) {
                    if ((cur.f0 & cur.f1) & WF_CLEAR) {
                        *reinterpret_cast<ulonglong2*>(sp) = make_ulonglong2(0ull, 0ull);
                        t_swr++;
                    } else if ((cur.f0 | cur.f1) & WF_CLEAR) {
                        sp[(cur.f0 & WF_CLEAR) ? 0 : 1] = 0ull;
                        t_swr++;
                    }
                    if (cur.pp_dirty) {
                        *reinterpret_cast<ulonglong2*>(fp) = make_ulonglong2(0ull, 0ull);
                        t_fwr++;
                    }
                } else {
                    t_srd++;
                    uint64_t n0 = acc0 & ~s2.x & k0;
                    uint64_t n1 = acc1 & ~s2.y & k1;
                    if (cur.f0 & WF_GROUP) n0 = group_fix(n0, s2.x, a.ctl[cur.w].gmask, a.ctl[cur.w].gstart);
                    if (cur.f1 & WF_GROUP) n1 = group_fix(n1, s2.y, a.ctl[cur.w + 1].gmask, a.ctl[cur.w + 1].gstart);
                    if ((n0 | n1) != 0ull || ((cur.f0 | cur.f1) & WF_CLEAR)) {
                        *reinterpret_cast<ulonglong2*>(sp) = make_ulonglong2(s2.x | n0, s2.y | n1);
                        t_swr++;
                    }
                    if ((n0 | n1) != 0ull || cur.pp_dirty) {
                        *reinterpret_cast<ulonglong2*>(fp) = make_ulonglong2(n0, n1);
                        t_fwr++;
                    }
                    cnt += (uint32_t)(__popcll(n0) + __popcll(n1));
                    if (a.snap) {
                        if (cur.f0 & WF_SNAP) snap_local += (unsigned long long)__popcll(n0 & a.ctl[cur.w].snap);
                        if (cur.f1 & WF_SNAP) snap_local += (unsigned long long)__popcll(n1 & a.ctl[cur.w + 1].snap);
                    }
                    if (a.use_lds) {
                        if (n0) atomicOr(&s_live[cur.w], (unsigned long long)n0);
                        if (n1) atomicOr(&s_live[cur.w + 1], (unsigned long long)n1);
                    } else {
                        if (n0) atomicOr(&a.live[cur.w], (unsigned long long)n0);
                        if (n1) atomicOr(&a.live[cur.w + 1], (unsigned long long)n1);
                    }
                }
            }
            // ---- per-node counters after the node's last pass ----
            if (cur.pass + 1u == npass) {
                uint32_t c = cnt;
#pragma unroll
                for (int off = GRP / 2; off > 0; off >>= 1) c += __shfl_xor(c, off, GRP);
                if (gl == 0 && c) {
                    a.recv[cur.v] += c;
                    a.sent[cur.v] += (uint64_t)c * a.deg[cur.v];
                }
                cnt = 0;
            }
            cur = nxt;
        }
    }
    if (a.snap) {
        snap_local = wave_sum(snap_local);
        if (lane == 0 && snap_local) atomicAdd(a.snap, snap_local);
    }
    if (a.acct) {
        t_pe = wave_sum(t_pe);
        t_col = wave_sum(t_col);
        t_srd = wave_sum(t_srd);
        t_swr = wave_sum(t_swr);
        t_fwr = wave_sum(t_fwr);
        if (lane == 0) {
            atomicAdd(&a.acct[0], t_pe);
            atomicAdd(&a.acct[1], t_col);
            atomicAdd(&a.acct[2], t_srd);
            atomicAdd(&a.acct[3], t_swr);
            atomicAdd(&a.acct[4], t_fwr);
        }
    }
    if (a.use_lds) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < a.wact; i += 256) {
            const unsigned long long x = s_live[i];
            if (x) atomicOr(&a.live[i], x);
        }
    }
}
