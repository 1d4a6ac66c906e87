// Batched 2D A* (and Dijkstra / GBFS) for gfx950, several queries per wave: bit-exact with the
// reference AStar.plan (global_planner/graph_search/a_star.py:39-83) including CPython heapq's tie
// behaviour (Lib/heapq.py heappush/_siftdown, heappop/_siftup) under Node.__lt__
// (utils/environment/node.py:51-54) -- the same algorithm as astar2d.hip, laid out differently.
//
// Why a second engine.  astar2d.hip runs one query per wave: every per-query value (heap size,
// sift path, root, last) is wave-uniform and lives in SGPRs, so the heap walk is scalar code.  The
// scalar unit is one per CU, shared by its 4 SIMDs, and the PMC issue breakdown of that kernel
// (profiles/r2/pmc_astar2d_issue.txt: 129 SALU + 112 VALU per heap operation) puts it at ~90 % of
// the per-SIMD scalar issue rate while the vector pipes idle at ~40 %.  Here a wave runs FOUR
// queries, one per 16-lane DPP row ("group"); every per-query value lives in VGPRs (equal across
// its row), so the walk, the compares and the placements are vector instructions serving four
// queries at once, and the scalar unit only runs the loop.  Cross-lane traffic stays inside a row:
// DPP row_newbcast (lane k of my row), DPP row_ror reductions, ds_bpermute for a variable lane, and
// 16-bit slices of ballots.
//
// Per group (query) state, identical in its 16 lanes: the query, the heap size n, heap[0] (root)
// and heap[n-1] (last) in registers, the pending pushes of the current expansion (a motion mask)
// and the parents of the positions those pushes take (prefetched with the expansion).
//
// The step (round 4): every group runs ONE heap operation per step -- a pop (with the 3x3 round and
// the expansion) when it has no pushes pending, else its next push -- in one code path for both
// (path_op): CPython's heappop and heappush are both a rotation of one root-to-node path, so a step
// costs one such operation whatever the mix.  The round-3 kernel ran every group's pop and then
// push rounds in lock step; 61 % of pops are stale and push nothing, so its 1.44 push rounds per
// iteration (a memory round trip each) left 64 % of the groups idle.  Alone the change was neutral
// (12.7 k plans/s either way: fewer waits, more scalar control); with 128 VGPRs it allows four waves
// per SIMD, and 56 queries resident per CU (128 LDS heap positions each) reach 16.4 k plans/s where
// the lock-step kernel lost throughput past 32.
//
// Heap storage per group: positions < lds_cap in LDS (f64 f[], u32 cm[] as SoA), the rest in a
// per-group HBM spill (16 B entries) read and written through one buffer descriptor per wave;
// CPython _siftup's child-choice ("direction") bits in 5-level blocks, tiers 0-1 in LDS and tier 2
// (levels 10-14) in LDS (T2LDS) or HBM.  Heaps are limited to kMqCap entries (levels 0-14); a
// query that outgrows it stops with PMP_CAP_OVERFLOW and the host re-runs it on astar2d.hip.
//
// Cell state: one byte per cell per group, (epoch << 4) | (parent motion + 1) for a CLOSED cell,
// where the epoch (1..15) numbers the group's queries, so a new query needs no reset of the 1 MiB
// array except every 15th query.  g of a CLOSED cell in a per-group f64 array (as astar2d.hip).
#include "pmp_internal.h"
#include "grid2d.h"

namespace {

constexpr double kSqrt2 = 1.4142135623730951;  // math.sqrt(2) == math.hypot(1, 1)
constexpr int kMqCap = 32767;                   // positions 0..32766: levels 0..14 (tier 2 in HBM)
constexpr int kMqCapT2L = 16383;                // positions 0..16382: levels 0..13 (tier 2 in LDS)
constexpr int kBits01 = 144;                    // LDS bytes of bit tiers 0-1 (33 words) per group
constexpr int kT2Words = 1024;                  // HBM tier-2 bit blocks (levels 10-14) per group
constexpr int kT2LBytes = 1024;                 // LDS tier-2 bit blocks (levels 10-12, 7 bits each) per group
constexpr int kMqLoneMax = 256;                 // batches up to this size: one query per wave (lone)

// motions in the order of env.py:52-55: (-1,0),(-1,1),(0,1),(1,1),(1,0),(1,-1),(0,-1),(-1,-1)
constexpr uint32_t kMx1 = 0x1A90u, kMy1 = 0x01A9u;
__device__ __forceinline__ int mot_x(int d) { return (int)((kMx1 >> (2 * d)) & 3u) - 1; }
__device__ __forceinline__ int mot_y(int d) { return (int)((kMy1 >> (2 * d)) & 3u) - 1; }

// HEUR bits 0-1: 0 euclidean, 1 manhattan (GraphSearcher.h, graph_search.py:41-44), 2 zero
// (Dijkstra); bit 2 (kThetaLayout): the Theta* entry layout of astar2d.hip -- a 5-bit code (0..7 the
// pusher's motion, 16 + motion "path 2": the parent is the pusher's own parent, theta_star.py:104-108;
// 8 the start) and a 13-bit dy (H <= 4096)
constexpr int kThetaLayout = 4;
template <int HEUR> constexpr int hkind() { return HEUR & 3; }
template <int HEUR> constexpr int dbits() { return (HEUR & kThetaLayout) ? 5 : 4; }
template <int HEUR>
__device__ __forceinline__ uint32_t pack_cm(int dx, int dy, int dir)
{
    constexpr int S = dbits<HEUR>();
    return ((uint32_t)dx << 18) | (((uint32_t)dy & ((1u << (18 - S)) - 1u)) << S) | (uint32_t)dir;
}
template <int HEUR> __device__ __forceinline__ int cm_dx(uint32_t cm) { return (int)cm >> 18; }
template <int HEUR> __device__ __forceinline__ int cm_dy(uint32_t cm) { return (int)(cm << 14) >> (14 + dbits<HEUR>()); }
template <int HEUR> __device__ __forceinline__ int cm_dir(uint32_t cm) { return (int)(cm & ((1u << dbits<HEUR>()) - 1u)); }
template <int HEUR>
__device__ __forceinline__ uint32_t hkey(uint32_t cm)
{
    if (hkind<HEUR>() == 2) return 0u;
    const int dx = cm_dx<HEUR>(cm), dy = cm_dy<HEUR>(cm);
    if (hkind<HEUR>() == 1) return (uint32_t)(abs(dx) + abs(dy));
    return (uint32_t)(__mul24(dx, dx) + __mul24(dy, dy));
}
template <int HEUR>
__device__ __forceinline__ double h_of_key(uint32_t hk)
{
    return hkind<HEUR>() == 2 ? 0.0 : (hkind<HEUR>() == 1 ? (double)hk : sqrt_int_rn(hk));
}
// Node.__lt__ (node.py:51-54)
__device__ __forceinline__ bool key_lt(double fa, uint32_t ka, double fb, uint32_t kb)
{
    return (fa < fb) | ((fa == fb) & (ka < kb));
}
// the same as a lane mask: three compares into SGPR pairs and two scalar ops (a ballot of the bool
// above would first turn it into a 0 / 1 VGPR and compare that again)
__device__ __forceinline__ lmask key_lt_m(double fa, uint32_t ka, double fb, uint32_t kb)
{
    return lm(fa < fb) | (lm(fa == fb) & lm(ka < kb));
}

// lane masks of the row positions (lane & 15) a predicate depends on
constexpr lmask kLanesGe1 = ~0x0001000100010001ull;  // gl >= 1
constexpr lmask kLane15 = 0x8000800080008000ull;     // gl == 15
constexpr lmask kLanesLt8 = 0x00FF00FF00FF00FFull;   // gl < 8
constexpr lmask kLanesLt9 = 0x01FF01FF01FF01FFull;   // gl < 9

typedef __attribute__((address_space(3))) double lds_f64;
typedef __attribute__((address_space(3))) uint32_t lds_u32;

// ---- row (16-lane group) primitives ----------------------------------------------------------
template <int K>
__device__ __forceinline__ uint32_t bc(uint32_t v)  // lane K of my row
{
    // mov_dpp (no `old` operand): every lane of a row_newbcast reads a valid lane, so no v_mov of a
    // fallback value is needed
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x150 + K, 0xF, 0xF, false);
}
template <int K>
__device__ __forceinline__ int bci(int v) { return (int)bc<K>((uint32_t)v); }
template <int K>
__device__ __forceinline__ double bcf(double v)
{
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    return __longlong_as_double(((uint64_t)bc<K>((uint32_t)(b >> 32)) << 32) | bc<K>((uint32_t)b));
}
__device__ __forceinline__ uint32_t shl1(uint32_t v)  // lane + 1 of my row (row_shl:1; lane 15 gets 0)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x101, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t shr1(uint32_t v)  // lane - 1 of my row (row_shr:1; lane 0 gets 0)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
}
__device__ __forceinline__ double shr1f(double v)
{
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    return __longlong_as_double(((uint64_t)shr1((uint32_t)(b >> 32)) << 32) | shr1((uint32_t)b));
}
__device__ __forceinline__ double shl1f(double v)
{
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    return __longlong_as_double(((uint64_t)shl1((uint32_t)(b >> 32)) << 32) | shl1((uint32_t)b));
}
__device__ __forceinline__ uint32_t ror_or(uint32_t v)  // OR over my row
{
    v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x121, 0xF, 0xF, false);
    v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x122, 0xF, 0xF, false);
    v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false);
    v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);
    return v;
}
// value of absolute lane `src` (same row), any src per lane
__device__ __forceinline__ uint32_t bp(uint32_t v, int src) { return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v); }
__device__ __forceinline__ double bpf(double v, int src)
{
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    return __longlong_as_double(((uint64_t)bp((uint32_t)(b >> 32), src) << 32) | bp((uint32_t)b, src));
}
// my row's 16 bits of a ballot
__device__ __forceinline__ uint32_t rbits(bool p, int gb) { return (uint32_t)(lm(p) >> gb) & 0xFFFFu; }

// per lane: bit `lane` of mask ? a : b, as one v_cndmask (see astar2d.hip Ld::get)
__device__ __forceinline__ uint32_t sel_lanes(uint64_t mask, uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %2, %1, %3" : "=v"(r) : "v"(a), "v"(b), "s"(mask));
    return r;
}
__device__ __forceinline__ void ds_mskor(lds_u32* w, uint32_t mask, uint32_t val)
{
    asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"((uint32_t)(uintptr_t)w), "v"(mask), "v"(val) : "memory");
}
__device__ __forceinline__ void wave_sync_mem() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// ---- heap storage of one group ------------------------------------------------------------------
struct GHeap {
    lds_f64* F;      // LDS f[cap]
    lds_u32* C;      // LDS cm[cap]
    lds_u32* K;      // LDS hkey[cap] (kKeys)
    lds_u32* B;      // LDS bit words: tier 0 (word 0), tier 1 (words 1..32)[, tier-2 bytes from word 36]
    uint32_t* T2;    // HBM tier-2 words (when not in LDS)
    __amdgpu_buffer_rsrc_t spill;  // the wave's spill region (4 groups)
    uint32_t sbase;  // byte offset of heap position 0 in the spill region (mod 2^32): positions >= cap are spilled
    uint32_t gbase;  // kBlocks: this group's byte offset in the wave's spill region
    int L0;          // kBlocks: level of position cap (the first level with spilled positions)
    int cap;
    __amdgpu_buffer_rsrc_t mirror;  // kMirror: the mirror of the wave's spill region
};
constexpr uint32_t kOOR = 0x80000000u;  // a buffer offset beyond any spill region: loads 0, stores dropped
#ifndef PMP_MQ_SPILL_SHIFT
#define PMP_MQ_SPILL_SHIFT 1
#endif
constexpr int kSpillShift = PMP_MQ_SPILL_SHIFT;  // empty slots in front of position cap
// Keep each entry's h order key (hkey) beside it: an LDS array (16 B per LDS position instead of 12)
// and the spill record's fourth word, so loaded entries need no key rebuild (A/B switch)
#ifndef PMP_MQ_KEYS
#define PMP_MQ_KEYS 0
#endif
constexpr bool kKeys = PMP_MQ_KEYS != 0;
constexpr int kEntLds = kKeys ? 16 : 12;  // LDS bytes per heap position
// Spill layout: two-level blocks (default): from level L0 (position cap's level) down, bands of two
// levels; the block of a node Q at the level above a band holds Q's two children and four
// grandchildren (6 x 16 B in one 128-B line), so a path and its siblings touch one line per two
// spilled levels instead of one per level (round 4, same-box A/B: 15.5 k -> 16.6-17.1 k plans/s,
// FETCH -18 %, WRITE -14 %).  Round 5 default (PMP_MQ_BLOCKS=2): each child with its own two
// children in one 64-B half of the block, so a rotation's two stores per band dirty one half
// (write-back sectors) instead of both -- WRITE -7 % at the same plans/s (profiles/r5/attribution.txt);
// 1: the round-4 order [c0 c1 g00 g01 g10 g11]; 0: position order, sibling pairs 32-B aligned.
#ifndef PMP_MQ_BLOCKS
#define PMP_MQ_BLOCKS 2
#endif
constexpr bool kBlocks = PMP_MQ_BLOCKS != 0;
constexpr bool kBlocks2 = PMP_MQ_BLOCKS == 2;
// Write-traffic attribution (dev builds only, tools/build_variant.sh): every store of the selected
// categories is issued twice, the copy into a mirror region with the same layout, so the extra
// WRITE_SIZE over the default build is that category's write traffic.  Bits: 1 the trivial-push run's
// spill stores, 2 a push rotation's spill stores, 4 a pop rotation's spill stores, 8 the cell-state
// byte and G of a closed cell (even slots only: the mirror of every slot's 9 MB would not fit beside
// the 15,360 slots' own, so that category's extra is doubled in the analysis).
#ifndef PMP_MQ_MIRROR
#define PMP_MQ_MIRROR 0
#endif
// path_op's level shift: ds_bpermute from the group's direction (1, default: +0.8 % plans/s on the
// VALU-bound step, three alternating rounds in tools/r5_call18.sh) or both DPP row shifts (0)
#ifndef PMP_MQ_BPERM
#define PMP_MQ_BPERM 1
#endif
constexpr int kMirror = PMP_MQ_MIRROR;
// Push pairs (round 6): a group whose next two pending pushes land at sibling positions (n, n + 1
// with n odd) runs both in one path operation -- the second _siftdown walks the same ancestors.
// Parity-green (tests/test_heap_path_form.py models it against heapq; the GPU suite passed with it
// on) but neutral on the headline: 19,129 vs 19,167 plans/s without (tools/calls/r6_call13.sh,
// interleaved): 7 % fewer path operations, each heavier, on a step that waits on memory.  Off.
#ifndef PMP_MQ_PAIR
#define PMP_MQ_PAIR 0
#endif
constexpr bool kPair = PMP_MQ_PAIR != 0;

// byte offset of spilled heap position p (>= cap) in the wave's spill region
__device__ __forceinline__ uint32_t spill_off(const GHeap& h, int p)
{
    if (!kBlocks) return h.sbase + (uint32_t)p * 16u;
    const uint32_t u = (uint32_t)p + 1u;
    const int lam = (31 - __clz((int)u)) - h.L0;  // level below L0 (>= 0 for a spilled position)
    const int o = lam & 1, b = lam >> 1;
    const uint32_t Q = u >> (o + 1);  // 1-based index of the block's node at the level above the band
    // blocks before band b: 2^(L0-1) (4^b - 1) / 3; band b's first node index 2^(L0+2b-1):
    // blk = Q - 2^(L0-1) (2 4^b + 1) / 3, and (2 4^b + 1) / 3 = 1, 3, 11, 43, 171 for b = 0..4
    const uint32_t kb = (uint32_t)(0xAB2B0B0301ull >> (8 * b)) & 0xFFu;
    const uint32_t blk = Q - (kb << (h.L0 - 1));
    // kBlocks 1: [c0 c1 g00 g01 g10 g11]; kBlocks 2: [c0 g00 g01 -][c1 g10 g11 -] (a child and its
    // two children in one 64-B half: a path writes one half of a block)
    const uint32_t slot = kBlocks2 ? (o ? ((u >> 1) & 1u) * 4u + 1u + (u & 1u) : (u & 1u) * 4u)
                                   : (u & ((2u << o) - 1u)) + 2u * (uint32_t)o;
    return h.gbase + blk * 128u + slot * 16u;
}

// The block layout's offset needs only the position's level below L0 (band b, parity o) besides the
// position itself; the level constants are fixed per launch, so lane L of a group holds those of heap
// level L (lane_cw, computed once) and a position at level K takes lane K's word (a DPP / bpermute,
// not ~20 VALU instructions of clz and 64-bit shifts): spill_off_cw.  A path operation's lanes hold
// the path's levels in order, so each uses its own word; a node's sibling sits in the next 16-B slot
// of the same block (offset ^ 16) -- with an odd LDS cap (GHeap.cap), sibling pairs never straddle
// the LDS / spill boundary.
#ifndef PMP_MQ_LANECONST
#define PMP_MQ_LANECONST 1
#endif
constexpr bool kLaneConst = PMP_MQ_LANECONST != 0 && kBlocks;
__device__ __forceinline__ uint32_t lane_cw(int L0, int level)
{
    const int lam = level - L0;
    if (lam < 0) return 0u;  // an LDS level: never used for an offset
    const int o = lam & 1, b = lam >> 1;
    const uint32_t kb = (uint32_t)(0xAB2B0B0301ull >> (8 * b)) & 0xFFu;
    return ((kb << (L0 - 1)) << 1) | (uint32_t)o;
}
__device__ __forceinline__ uint32_t spill_off_cw(const GHeap& h, uint32_t cw, int p)
{
    const uint32_t u = (uint32_t)p + 1u;
    const uint32_t o = cw & 1u;
    const uint32_t blk = (u >> (o + 1u)) - (cw >> 1);
    const uint32_t slot = kBlocks2 ? (o ? ((u >> 1) & 1u) * 4u + 1u + (u & 1u) : (u & 1u) * 4u)
                                   : (u & ((2u << o) - 1u)) + 2u * o;
    return h.gbase + (blk << 7) + (slot << 4);
}
// the sibling's offset: the next slot of the pair (kBlocks 1: slots 2i, 2i + 1), or the other half's
// child / the pair 4i + 1, 4i + 2 (kBlocks 2)
__device__ __forceinline__ uint32_t sib_xor(uint32_t cw) { return kBlocks2 ? ((cw & 1u) ? 48u : 64u) : 16u; }

struct Ld {
    double fl;
    uint32_t cl, kl;
    uint4 v;
    bool in;
    __device__ __forceinline__ void issue(const GHeap& h, int p) { issue_off(h, p, p < h.cap ? kOOR : spill_off(h, p)); }
    // off: the spill offset of p when p >= cap (else ignored)
    __device__ __forceinline__ void issue_off(const GHeap& h, int p, uint32_t off)
    {
        in = p < h.cap;
        const int pl = in ? p : 0;
        v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(h.spill, in ? kOOR : off, 0, 0));
        fl = h.F[pl];
        cl = h.C[pl];
        if (kKeys) kl = h.K[pl];
    }
    // the entry (f, code) and its h order key
    template <int HEUR>
    __device__ __forceinline__ void get(double& f, uint32_t& c, uint32_t& k) const
    {
        const uint64_t m = __ballot(in);
        const uint64_t b = (uint64_t)__double_as_longlong(fl);
        f = __hiloint2double((int)sel_lanes(m, (uint32_t)(b >> 32), v.y), (int)sel_lanes(m, (uint32_t)b, v.x));
        c = sel_lanes(m, cl, v.z);
        k = kKeys ? sel_lanes(m, kl, v.w) : hkey<HEUR>(c);
    }
};
__device__ __forceinline__ void hst_off(const GHeap& h, bool on, int p, uint32_t soff, double f, uint32_t c, uint32_t k,
                                        int cat = 0)
{
    if (on && p < h.cap) {
        h.F[p] = f;
        h.C[p] = c;
        if (kKeys) h.K[p] = k;
    }
    const uint64_t b = (uint64_t)__double_as_longlong(f);
    const uint4 v = make_uint4((uint32_t)b, (uint32_t)(b >> 32), c, kKeys ? k : 0u);
    const uint32_t off = (on && p >= h.cap) ? soff : kOOR;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v),
                                           h.spill, off, 0, 0);
    if (kMirror & cat)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v),
                                               h.mirror, off, 0, 0);
}
__device__ __forceinline__ void hst(const GHeap& h, bool on, int p, double f, uint32_t c, uint32_t k, int cat = 0)
{
    hst_off(h, on, p, (on && p >= h.cap) ? spill_off(h, p) : kOOR, f, c, k, cat);
}

// ---- direction bits (astar2d.hip: bit(p) = !(heap[2p+1] < heap[2p+2]) for nodes with two children,
// 5-level blocks; node Pl (path number) at level L: tier t = L / 5, r = L - 5t, block root R = Pl >> r,
// bit (Pl & (2^r - 1)) + 2^r - 1 of the block word).  With the tier-2 blocks in LDS (T2LDS) heaps stop
// at level 13, so tier 2 only holds the bits of levels 10-12: 7 bits per block, one byte each.
//
// A walk through a block is found without a dependent chain: the bits define exactly one leaf whose
// path they agree with, so each lane tests two candidate leaves of a 5-level block (one of a 3-level
// block) against masks fixed per lane (Walk), and the row's ballot names the leaf.
struct Walk {
    uint32_t MA, VA, MB, VB, MV3;  // leaves gl and gl + 16 of a 5-level block; leaf gl & 7 of a 3-level one (M | V << 8)
    __device__ __forceinline__ static void leaf(int L, int lev, uint32_t& M, uint32_t& V)
    {
        uint32_t pr = 1;
        M = V = 0u;
        for (int k = 0; k < lev; k++) {
            const uint32_t b = (uint32_t)(L >> (lev - 1 - k)) & 1u;
            M |= 1u << pr;
            V |= b << pr;
            pr = 2u * pr + b;
        }
    }
    __device__ __forceinline__ void init(int gl)
    {
        leaf(gl, 5, MA, VA);
        leaf(gl + 16, 5, MB, VB);
        uint32_t M3, V3;
        leaf(gl & 7, 3, M3, V3);
        MV3 = M3 | (V3 << 8);
    }
    // path number (block-relative) after five / three steps from the block root; w2 = block word << 1
    __device__ __forceinline__ uint32_t five(uint32_t w2, int gb) const
    {
        const uint32_t a = rbits((w2 & MA) == VA, gb), b = rbits((w2 & MB) == VB, gb);
        return 32u + (uint32_t)__builtin_ctz(a | (b << 16));  // exactly one leaf matches: never 0
    }
    __device__ __forceinline__ uint32_t three(uint32_t w2, int gb) const
    {
        return 8u + (uint32_t)__builtin_ctz(rbits((w2 & MV3 & 0xFFu) == (MV3 >> 8), gb) & 0xFFu);
    }
};
template <bool T2LDS>
__device__ __forceinline__ uint32_t t2_load(const GHeap& h, uint32_t R2)
{
    if (T2LDS) {
        const uint32_t b = R2 - 1024u;
        return (h.B[36u + (b >> 2)] >> (8u * (b & 3u))) & 0x7Fu;
    }
    return __hip_atomic_load(h.T2 + (R2 - 1024u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// set (on lanes with `on`) the bit of node Pl at `level` to `bit`
template <bool T2LDS>
__device__ __forceinline__ void bit_set(const GHeap& h, bool on, int level, uint32_t Pl, bool bit)
{
    const int t = (int)((uint32_t)__mul24(level, 13) >> 6);  // level / 5 for level < 64
    const int r = level - 5 * t;
    const uint32_t mr = (1u << r) - 1u;
    const uint32_t R = Pl >> r;
    uint32_t m = 1u << ((Pl & mr) + mr);
    if (T2LDS) {  // every tier in LDS: one masked write at a computed word, no branch per tier
        const uint32_t b2 = R - 1024u;
        const uint32_t widx = t == 0 ? 0u : (t == 1 ? R - 31u : 36u + (b2 >> 2));
        m = t == 2 ? m << (8u * (b2 & 3u)) : m;
        if (on) ds_mskor(h.B + widx, m, bit ? m : 0u);
        return;
    }
    if (!on) return;
    if (t == 0) {
        ds_mskor(h.B, m, bit ? m : 0u);
    } else if (t == 1) {
        ds_mskor(h.B + (R - 31u), m, bit ? m : 0u);
    } else {
        uint32_t* w = h.T2 + (R - 1024u);
        if (bit) __hip_atomic_fetch_or(w, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else __hip_atomic_fetch_and(w, ~m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
// path_op's form: lane L (1..15) sets the bit of its parent, node Pl at level L - 1, so each lane's
// tier is a compile-time lane mask (levels 0-4 / 5-9 / 10-14 at lanes 1-5 / 6-10 / 11-15) and, with
// the tier-2 bytes in LDS, the word is one shift and add: tier 0's block root is 1 (word 0), tier 1's
// 32..63 (words 1..32), tier 2's 1024..2047 (bytes from word 36).  Only heaps of <= 16,383 entries
// (T2LDS) use it; the HBM tier-2 form keeps bit_set.
constexpr lmask kTier1 = 0x07C007C007C007C0ull;  // gl 6..10
constexpr lmask kTier2 = 0xF800F800F800F800ull;  // gl 11..15
__device__ __forceinline__ void bit_set_lane(const GHeap& h, bool on, int gl, uint32_t Pl, bool bit)
{
    const bool t1 = lb(kTier1), t2 = lb(kTier2);
    const int r = gl - 1 - (t2 ? 10 : (t1 ? 5 : 0));  // level - 5 t
    const uint32_t R = Pl >> r;
    const uint32_t mr = (1u << r) - 1u;
    const uint32_t widx = t2 ? (R >> 2) - 220u : (t1 ? R - 31u : R - 1u);
    const uint32_t m = 1u << ((Pl & mr) + mr + (t2 ? (R & 3u) << 3 : 0u));
    if (on) ds_mskor(h.B + widx, m, bit ? m : 0u);
}
// CPython _siftup's choice bit of the parent of `child` (a position) whose new content is v and
// whose sibling holds s: bit = !(left < right), odd positions are left children
__device__ __forceinline__ bool choice_bit_k(int child, double vf, uint32_t vk, double sf, uint32_t sk)
{
    return (child & 1) ? !key_lt(vf, vk, sf, sk) : !key_lt(sf, sk, vf, vk);
}
// ---- the step ---------------------------------------------------------------------------------
// Each step every group runs ONE heap operation: a pop (with the 3x3 round and the expansion) when
// it has no pushes pending, else the next pending push; the leading run of trivial pushes is stored
// first in the same step (and a group whose run empties its pushes pops in that step).  A group's
// pop and push are one path operation of the same code (path_op), so a step costs about one such
// operation and every group advances in it (tests/test_heap_path_form.py checks the path form
// against Lib/heapq).

// _siftup's leaf for a heappop on a heap of n (> 0) entries: path number P (1-based) and level K
template <bool T2LDS>
__device__ __forceinline__ void pop_leaf(const GHeap& h, const Walk& wk, int n, int gb, uint32_t& P, int& K)
{
    const int D = 31 - __clz(n);
    const int full = D - 1 < 0 ? 0 : D - 1;
    const uint32_t w0 = h.B[0] << 1;
    const uint32_t pr0 = wk.five(w0, gb);  // level-5 node (32..63) along the tier-0 bits
    uint32_t w1 = 0u, w2 = 0u, pr1 = 32u, pr2 = T2LDS ? 8u : 32u;
    if (full >= 5) {
        w1 = h.B[pr0 - 31u] << 1;
        pr1 = wk.five(w1, gb);
    }
    const uint32_t R2 = (pr0 << 5) + pr1 - 32u;  // level-10 node (1024..2047)
    if (full >= 10) {
        w2 = t2_load<T2LDS>(h, R2) << 1;
        pr2 = T2LDS ? wk.three(w2, gb) : wk.five(w2, gb);
    }
    const int tf = full >= 10 ? 2 : (full >= 5 ? 1 : 0);
    const int rf = full - 5 * tf;
    const uint32_t wt = tf == 2 ? w2 : (tf == 1 ? w1 : w0);
    const uint32_t prt = tf == 2 ? pr2 : (tf == 1 ? pr1 : pr0);
    const uint32_t Rt = tf == 2 ? R2 : (tf == 1 ? pr0 : 1u);
    const uint32_t prel = prt >> ((tf == 2 && T2LDS ? 3 : 5) - rf);
    P = (Rt << rf) + prel - (1u << rf);
    K = D - 1 < 0 ? 0 : D - 1;
    if (2u * P <= (uint32_t)n) {
        const uint32_t c = (2u * P < (uint32_t)n) ? ((wt >> prel) & 1u) : 0u;
        P = 2u * P + c;
        K++;
    }
}

// One heap operation of a group on the path q_L = (Q >> (Kd - L)) - 1, L = 0..Kd (lane L <-> level L):
//  pop  (heap already shrunk to n; X = the old last element; the path = _siftup's, root to leaf):
//       the prefix of levels 1..b with !(X < heap[q_L]) moves up one level, X lands at level b;
//  push (X = the item at position n = q_Kd; the path = its ancestors, _siftdown): the levels
//       b..Kd-1 with X < heap[q_L] move down one level, X lands at level b.
// One load round (lane L: heap[q_L] and its sibling; lane 15 of a pop: heap[n - 1], the new last),
// a ballot for b, the stores, the bits of the changed levels' parents.  Returns b; lane L's new
// heap[q_L] in (nf, nc, nk) (for the caller's cached parents).
template <bool T2LDS, int HEUR>
__device__ __forceinline__ int path_op(const GHeap& h, lmask mon, lmask mpop, uint32_t Q, int Kd, int n, double Xf, uint32_t Xc,
                                       uint32_t Xk, int gl, int gb, double& lastf, uint32_t& lastc, uint32_t& lastk,
                                       double& rootf, uint32_t& rootc, double& nf, uint32_t& nc, uint32_t& nk, uint32_t cwL,
                                       lmask mpair = 0ull, double X2f = 0.0, uint32_t X2c = 0u, uint32_t X2k = 0u)
{
    // the lane predicates as lane masks (scalar logic, lm / lb): the step is VALU-issue-bound
    const bool lvl = gl <= Kd;
    const int q = lvl ? (int)(Q >> (Kd - gl)) - 1 : 0;
    const bool on = lb(mon), pop = lb(mpop);
    const lmask mlvl = lm(lvl);
    const lmask mlda = mon & ((mpop & mlvl & kLanesGe1) | (~mpop & lm(gl < Kd)));
    const bool lda = lb(mlda);
    const bool l15 = lb(mon & mpop & kLane15);  // a pop's lane 15: heap[n - 1], the new last
    const bool p15 = kPair && lb(mpair & kLane15);  // a push pair's lane 15: the second leaf, position n + 1
    const int si = ((q - 1) ^ 1) + 1;
    const lmask mhass = mon & kLanesGe1 & mlvl & lm(si < n);
    const bool hass = lb(mhass);
    double Vf, Sf;
    uint32_t Vc, Sc, Vk, Sk;
    // kLaneConst: one offset per lane -- lane L's level-L word for the path node q (lane 15 of a pop:
    // the word of heap[n - 1]'s level, from that level's lane); the sibling is the next slot (^ 16);
    // the stores go to q, at the same offset (every storing lane loaded its q)
    uint32_t offq = kOOR;
    {
        Ld la, ls;
        if (kLaneConst) {
            const uint32_t cwK = bp(cwL, gb + (p15 ? Kd : 31 - __clz(n > 0 ? n : 1)));
            // the offset of q (of n - 1 on a pop's lane 15, which stores nothing; of n + 1, the pair's
            // second leaf, on a pair's lane 15); only the lanes whose value the operation uses load
            offq = spill_off_cw(h, (l15 || p15) ? cwK : cwL, l15 ? n - 1 : (p15 ? n + 1 : q));
            la.issue_off(h, lda ? q : (l15 ? n - 1 : 0), offq);
            ls.issue_off(h, hass ? si : 0, offq ^ sib_xor(cwL));
        } else {
            la.issue(h, lda ? q : (l15 ? n - 1 : 0));
            ls.issue(h, hass ? si : 0);
        }
        la.get<HEUR>(Vf, Vc, Vk);
        ls.get<HEUR>(Sf, Sc, Sk);
    }
    // the boundary level b
    const int cnt = __popc((uint32_t)((mlda & (mpop ^ key_lt_m(Xf, Xk, Vf, Vk))) >> gb) & 0xFFFFu);  // pop: !lt, push: lt
    const int b = pop ? cnt : Kd - cnt;
    // new contents: a pop shifts levels 1..b up one (lane L takes lane L+1's), a push shifts levels
    // b..Kd-1 down one (lane L takes lane L-1's); X at level b
    const lmask mblt = lm(gl < b), mbeq = lm(gl == b), mbgt = lm(gl > b);
    const bool atb = lb(mbeq), shift = lb((mpop & mblt) | (~mpop & mbgt & mlvl));
    // the levels a pop (<= b) / a push (>= b) rewrites
    const lmask mchg = (mpop & (mblt | mbeq)) | (~mpop & (mbgt | mbeq));
#if PMP_MQ_BPERM
    // one ds_bpermute per word from lane L +- 1 (the group's own direction) instead of both DPP
    // shifts and a select: the kernel is VALU-issue-bound, the permutes run on the LDS pipe.  A
    // shifting lane's source stays in its row (a pop shifts levels < b <= 14, a push levels > b >= 0)
    {
        const int sa = ((int)__lane_id() + (pop ? 1 : -1)) << 2;
        const uint64_t vb = (uint64_t)__double_as_longlong(Vf);
        const uint32_t flo = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)(uint32_t)vb);
        const uint32_t fhi = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)(uint32_t)(vb >> 32));
        const uint32_t shc = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)Vc);
        const uint32_t shk = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)Vk);
        const double shf = __longlong_as_double(((uint64_t)fhi << 32) | flo);
        nf = atb ? Xf : (shift ? shf : Vf);
        nc = atb ? Xc : (shift ? shc : Vc);
        nk = atb ? Xk : (shift ? shk : Vk);
    }
#else
    const double upf = shl1f(Vf), dnf = shr1f(Vf);
    const uint32_t upc = shl1(Vc), upk = shl1(Vk), dnc = shr1(Vc), dnk = shr1(Vk);
    nf = atb ? Xf : (shift ? (pop ? upf : dnf) : Vf);
    nc = atb ? Xc : (shift ? (pop ? upc : dnc) : Vc);
    nk = atb ? Xk : (shift ? (pop ? upk : dnk) : Vk);
#endif
    // ---- a push pair: the second item X2 goes in at position n + 1, the sibling of the first's, so
    // CPython's _siftdown walks the same ancestors, which now hold the first push's result: X2 lands
    // at the top of the chain's run of levels greater than it (b2 <= Kd - 1; the chain is ordered),
    // those levels move down one, and the chain's old bottom (or X2 itself, cnt2 = 0) becomes the
    // new leaf, which lane 15 holds and stores.  The first leaf stays on lane Kd.
    int bst = b;  // the first level the operation rewrote
    lmask mchg2 = mchg;
    if (kPair && mpair) {
        const int cnt2 = __popc((uint32_t)((mpair & lm(gl < Kd) & key_lt_m(X2f, X2k, nf, nk)) >> gb) & 0xFFFFu);
        const int b2 = Kd - cnt2;
        // lane L takes lane L - 1's chain value (L > b2), lane 15 the chain's bottom (lane Kd - 1);
        // gl = 0 never shifts (b2 >= 0), so its wrapped source is never used
        const int src2 = gb + (gl == 15 ? Kd - 1 : gl - 1);
        const double shf2 = bpf(nf, src2);
        const uint32_t shc2 = bp(nc, src2), shk2 = bp(nk, src2);
        const bool at2 = lb(mpair & lm(gl == b2) & lm(gl < Kd)) || (p15 && cnt2 == 0);
        const bool sh2 = lb(mpair & lm(gl > b2) & lm(gl < Kd)) || (p15 && cnt2 > 0);
        nf = at2 ? X2f : (sh2 ? shf2 : nf);
        nc = at2 ? X2c : (sh2 ? shc2 : nc);
        nk = at2 ? X2k : (sh2 ? shk2 : nk);
        if (lb(mpair)) bst = b2 < b ? b2 : b;
        mchg2 = (mchg & ~mpair) | (mpair & lm(gl >= bst));
    }
    const bool stq = lb((mon & mchg2 & mlvl) | (kPair ? mpair & kLane15 : 0ull));
    const int qs = p15 ? n + 1 : q;
    if (kLaneConst) hst_off(h, stq, qs, offq, nf, nc, nk, pop ? 4 : 2);
    else hst(h, stq, qs, nf, nc, nk, pop ? 4 : 2);
    // the bits of the changed levels' parents: lane L (>= 1) sets its parent's from its new content
    // and its sibling's: bit = !(left < right), an odd position is the left child (choice_bit_k)
    {
        lmask mbit = mhass & mchg2;
        if (kPair && mpair) {
            // a pair's first leaf (lane Kd, a left child) has the second leaf (lane 15) as its sibling
            const double lf2 = bpf(nf, gb + 15);
            const uint32_t lk2 = bp(nk, gb + 15);
            const lmask mkd = mpair & lm(gl == Kd);
            Sf = lb(mkd) ? lf2 : Sf;
            Sk = lb(mkd) ? lk2 : Sk;
            mbit |= mkd;
        }
        const bool fe = nf == Sf;
        const lmask lt_ns = lm(nf < Sf) | (lm(fe) & lm(nk < Sk));
        const lmask lt_sn = lm(nf > Sf) | (lm(fe) & lm(nk > Sk));
        const lmask modd = lm((q & 1) != 0);
        const bool bit = lb((modd & ~lt_ns) | (~modd & ~lt_sn));
        if (T2LDS) bit_set_lane(h, lb(mbit), gl, Q >> (Kd - gl + 1), bit);
        else bit_set<T2LDS>(h, lb(mbit), gl - 1, Q >> (Kd - gl + 1), bit);
    }
    {
        // selects, not a branch (every lane computes them): root = level 0's new content; the last
        // element: a pop's heap[n - 1] unless X landed on it (the path's leaf, b == Kd); a push's new
        // heap[n] (level Kd)
        const double r0f = bcf<0>(nf);
        const uint32_t r0c = bc<0>(nc);
        const int src = gb + ((pop || p15 || (kPair && lb(mpair))) ? 15 : Kd);
        const double lf = bpf(pop ? Vf : nf, src);
        const uint32_t lc = bp(pop ? Vc : nc, src), lk = bp(pop ? Vk : nk, src);
        const bool setl = lb(mon & ~(mpop & lm(b == Kd && Q == (uint32_t)n)));
        rootf = on ? r0f : rootf;
        rootc = on ? r0c : rootc;
        lastf = setl ? lf : lastf;
        lastc = setl ? lc : lastc;
        lastk = setl ? lk : lastk;
    }
    wave_sync_mem();
    return bst;
}

// THETA: 1 = ThetaStar (theta_star.py:44-108), 2 = LazyThetaStar (lazy_theta_star.py:38-114), with
// HEUR's Theta* layout bit; the CLOSED parent of a cell (any cell) per slot in Pc_all.
template <int HEUR, bool GZERO, bool T2LDS, int THETA = 0>
// <= 128 VGPRs: four waves per SIMD, up to 64 queries resident per CU (Theta*: three, the line-of-sight
// state would spill at 128)
// Theta* variants: 3 waves per SIMD (no scratch; a 128-VGPR build spills 20-60 B and was no faster,
// profiles/r5/theta_residency.txt)
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(THETA ? 3 : 4))) void astar2d_mqu_kernel(
    const uint32_t* __restrict__ occ, int W, int H, const int32_t* __restrict__ start_xy,
    const int32_t* __restrict__ goal_xy, const int32_t* __restrict__ order, int nq, double* __restrict__ cost_out,
    int32_t* __restrict__ path_len_out, uint32_t* __restrict__ path_out, int path_cap,
    int32_t* __restrict__ nexp_out, uint32_t* __restrict__ expand_out, int expand_cap,
    int64_t* __restrict__ counters, int32_t* __restrict__ status_out, int* __restrict__ queue,
    uint4* __restrict__ spill_all, int spill_n, int heap_cap, int lds_cap, int region, uint8_t* __restrict__ cst_all,
    size_t cst_bytes, double* __restrict__ G_all, uint32_t* __restrict__ t2_all, uint32_t* __restrict__ epoch_all,
    int prio_n, int lone, unsigned long long* __restrict__ span, uint32_t* __restrict__ Pc_all)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = lane_id();
    const int gl = lane & 15, gb = lane & 48, grp = lane >> 4;
    const size_t slot = (size_t)blockIdx.x * 4u + (size_t)grp;
    span_begin(span);
    GHeap hp;
    {
        // lone: group 0 alone, with the wave's whole LDS (the other groups retire at once and alias it)
        unsigned char* base = smem + (lone ? (size_t)0 : (size_t)grp * (size_t)region);
        hp.B = (lds_u32*)base;
        const int bits_b = T2LDS ? kBits01 + kT2LBytes : kBits01;
        hp.F = (lds_f64*)(base + bits_b);
        hp.C = (lds_u32*)(base + bits_b + (size_t)8 * lds_cap);
        hp.K = (lds_u32*)(base + bits_b + (size_t)12 * lds_cap);
        hp.T2 = t2_all + slot * kT2Words;
        hp.spill = __builtin_amdgcn_make_buffer_rsrc(spill_all + (size_t)blockIdx.x * 4u * (size_t)spill_n, 0,
                                                     (int)(4u * (uint32_t)spill_n * 16u), 0x00020000);
        hp.sbase = (uint32_t)grp * (uint32_t)spill_n * 16u + (uint32_t)(kSpillShift - lds_cap) * 16u;
        hp.gbase = (uint32_t)grp * (uint32_t)spill_n * 16u;
        hp.L0 = 31 - __clz(lds_cap + 1);
        // kLaneConst: an odd cap (one LDS slot unused), so no sibling pair straddles LDS and spill
        hp.cap = kLaneConst ? lds_cap - 1 : lds_cap;
        if (kMirror & 7)
            hp.mirror = __builtin_amdgcn_make_buffer_rsrc(
                spill_all + ((size_t)gridDim.x + blockIdx.x) * 4u * (size_t)spill_n, 0,
                (int)(4u * (uint32_t)spill_n * 16u), 0x00020000);
    }
    uint8_t* cst = cst_all + slot * cst_bytes;
    const size_t gsc = g_slot_cells(W, H);  // G: tiled (g_idx), slot stride gsc cells
    const uint32_t tHg = g_tiles_y(H);
    double* G = G_all + slot * gsc;
    // Theta*: G and Pc in 4 x 4 tiles (g_idx); A* keeps row-major G (the tile index cost the headline's
    // dependent chain 1.3 %, tools/calls/r6_call42.sh)
    auto gix = [&](int gx_, int gy_) -> uint32_t {
        return THETA ? g_idx(gx_, gy_, tHg) : (uint32_t)gx_ * (uint32_t)H + (uint32_t)gy_;
    };
    uint32_t* Pc = THETA ? Pc_all + slot * gsc : nullptr;  // CLOSED parent cell (linear), tiled like G
    const size_t nslots = (size_t)gridDim.x * 4u;
    const bool mir8 = (kMirror & 8) && (slot & 1u) == 0u;
    uint8_t* cst_m = cst_all + (nslots + slot / 2) * cst_bytes;
    double* G_m = G_all + (nslots + slot / 2) * gsc;

    Walk wk;
    wk.init(gl);
    const uint32_t cwL = kLaneConst ? lane_cw(hp.L0, gl) : 0u;  // spill-offset word of heap level gl
    // a spilled position p's offset from its level's word (lane gb + level of p)
    auto soff = [&](int p, bool on) -> uint32_t {
        if (!kLaneConst) return (on && p >= hp.cap) ? spill_off(hp, p) : kOOR;
        const uint32_t cw = bp(cwL, gb + (31 - __clz(p + 1)));
        return spill_off_cw(hp, cw, p);
    };
    // per-lane constants: lane m < 8 of a row is motion m (offset, cost, isCollision's cells)
    const int mo = gl & 7;
    const int mx = mot_x(mo), my = mot_y(mo);
    // need (the 3x3 cells isCollision wants free) | the motion's own cell << 16, one register
    uint32_t nsb = 16u | (1u << ((mx + 1) * 3 + (my + 1)));
    if (mo & 1) nsb |= (1u << (3 + (my + 1))) | (1u << ((mx + 1) * 3 + 1));
    nsb |= (1u << ((mx + 1) * 3 + (my + 1))) << 16;
    // the 3x3 round: lanes 0..8 the occupancy and the cell-state byte of cell (x + i/3 - 1,
    // y + i%3 - 1) (tiled cell states, cst_idx); lane 12 G[pusher]; THETA: lane 13 the pusher's CLOSED parent
    const int blk_dx = gl < 9 ? gl / 3 - 1 : 0;
    const int blk_dy = gl < 9 ? gl % 3 - 1 : 0;
    const uint32_t tH = cst_tiles_y(H);

    // group state (equal across the row)
    uint32_t ep = epoch_all[slot];
    // per-group flags as lane masks (SGPR pairs, scalar logic): a group needs a query / is done
    lmask Mneed = ~0ull, Mdone = lone ? lm(grp != 0) : 0ull;
    int q = 0, qi = 0, sx = 0, sy = 0, gx = 0, gy = 0;
    int n = 0, nexp = 0, maxn = 0;
    int npush = 0, npop = 0;  // < 2^31 per query (heaps are capped at 32,767 entries: pushes <= 8 W H)
    double rootf = 0.0, lastf = 0.0;
    uint32_t rootc = 0u, lastc = 0u, lastk = 0u;  // lastk = hkey(lastc)
    // the pushes of the last expansion still to do (motion mask, in motion order) and their items
    // (lane m < 8: motion m); lanes 0..7 hold heap[parent(n0 + lane)] while pc_ok
    uint32_t pend = 0u;
    double ifv = 0.0;
    uint32_t icm = 0u, ikk = 0u;
    lmask Mpc = 0ull;  // the group's cached parents (pf8, pk8) are valid ("pc_ok")
    double pf8 = 0.0;
    uint32_t pk8 = 0u;
    int n0 = 0;

    for (;;) {
        // ---- groups without a query take the next one (or retire)
        const lmask mfetch = Mneed & ~Mdone;
        if (lb(mfetch)) {
            int v = 0;
            if (gl == 0) v = atomicAdd(queue, 1);
            qi = bci<0>(v);
            if (qi < nq) {
                q = order ? order[qi] : qi;
                sx = start_xy[2 * q];
                sy = start_xy[2 * q + 1];
                gx = goal_xy[2 * q];
                gy = goal_xy[2 * q + 1];
                const bool s_in = (unsigned)sx < (unsigned)W && (unsigned)sy < (unsigned)H;
                const bool g_in = (unsigned)gx < (unsigned)W && (unsigned)gy < (unsigned)H;
                if (!s_in || !g_in) {  // outside the grid: blocked -> no neighbours -> no path
                    if (gl == 0) {
                        status_out[q] = PMP_NO_PATH;
                        cost_out[q] = 0.0;
                        path_len_out[q] = 0;
                        nexp_out[q] = s_in ? 1 : 0;
                        if (counters) {
                            counters[4 * q] = 1; counters[4 * q + 1] = 1;
                            counters[4 * q + 2] = s_in ? 1 : 0; counters[4 * q + 3] = 1;
                        }
                    }
                } else {
                    // next epoch; every 15th query (and a fresh slot, epoch 0) clears the cell states
                    if (ep == 0u || ep >= 15u) {
                        uint4* c4 = reinterpret_cast<uint4*>(cst);
                        const size_t n4 = cst_bytes / 16;
                        for (size_t i = gl; i < n4; i += 16) c4[i] = make_uint4(0u, 0u, 0u, 0u);
                        ep = 1u;
                    } else {
                        ep++;
                    }
                    // heap[0] = Node(start, start, 0, 0), key (0, h = 0)
                    rootf = 0.0;
                    rootc = pack_cm<HEUR>(0, 0, 8);
                    lastf = rootf;
                    lastc = rootc;
                    lastk = hkey<HEUR>(rootc);
                    hst(hp, gl == 0, 0, rootf, rootc, lastk);
                    n = 1;
                    npush = 1;
                    npop = 0;
                    nexp = 0;
                    maxn = 1;
                    pend = 0u;
                }
            }
            wave_sync_mem();
        }
        if (mfetch) {
            // the fetch's outcome (compares on every lane, kept to the fetching groups): the queue ran
            // out, or a query inside the grid started
            const lmask mend = mfetch & lm(qi >= nq);
            const lmask mstart = mfetch & ~mend & lm((unsigned)sx < (unsigned)W) & lm((unsigned)sy < (unsigned)H) &
                                 lm((unsigned)gx < (unsigned)W) & lm((unsigned)gy < (unsigned)H);
            Mdone |= mend;
            Mneed &= ~mstart;
            Mpc &= ~mstart;
            // the longest queries (first in the longest-first order) get issue priority
            if (~Mdone & ~Mneed & lm(qi < prio_n)) __builtin_amdgcn_s_setprio(3);
            else __builtin_amdgcn_s_setprio(0);
        }
        if (Mdone == ~0ull) break;
        const lmask Mact = ~Mdone & ~Mneed;

        // ---- 1. the leading run of trivial pushes (the item is not less than its parent, so
        //      CPython's _siftdown stops at once): stored in one step
        if (lb(Mact & Mpc & lm(pend != 0u))) {
            const uint32_t mine = (pend >> mo) & 1u;  // lane m < 8: my item is pending
            const uint32_t below = pend & ((1u << mo) - 1u);
            const int rank = __popc(below);
            const int pos = n + rank;
            const int pl = gb + (pos - n0 < 8 ? pos - n0 : 7);
            const double pf = bpf(pf8, pl);
            const uint32_t pk = bp(pk8, pl);
            const lmask mtriv = kLanesLt8 & lm(mine != 0u) & ~key_lt_m(ifv, ikk, pf, pk);
            const uint32_t tm = (uint32_t)(mtriv >> gb) & 0xFFu;
            const uint32_t nt = pend & ~tm;
            const uint32_t run = nt ? pend & ((nt & (0u - nt)) - 1u) : pend;
            if (run != 0u) {
                // heap[pos] = item; a right child sets its parent's bit against its left sibling (the
                // previous item of the run, or `last`)
                const bool inrun = gl < 8 && ((run >> mo) & 1u);
                const int prev = below ? 31 - __clz(below) : 0;
                const double lfp = bpf(ifv, gb + prev);
                const uint32_t lkp = bp(ikk, gb + prev);
                const double leftf = rank == 0 ? lastf : lfp;
                const uint32_t leftk = rank == 0 ? lastk : lkp;
                bit_set<T2LDS>(hp, lb(lm(inrun) & lm((pos & 1) == 0) & lm(pos > 0)), 30 - __clz(pos + 1),
                               (uint32_t)(pos + 1) >> 1, lb(~key_lt_m(leftf, leftk, ifv, ikk)));
                hst_off(hp, inrun, pos, soff(pos, inrun), ifv, icm, ikk, 1);
                const int top = 31 - __clz(run);
                lastf = bpf(ifv, gb + top);
                lastc = bp(icm, gb + top);
                lastk = bp(ikk, gb + top);
                const int k = __popc(run);
                n += k;
                npush += k;
                pend &= ~run;
                wave_sync_mem();
            }
        }

        // ---- 2. this step's heap operation: the next pending push, else a pop
        const lmask Mpush = Mact & lm(pend != 0u);
        const bool push = lb(Mpush);
        int st = -1;  // >= 0: the query ends this step with this status
        double goal_cost = 0.0;
        int plen = 0;
        if (lb(Mact & ~Mpush & lm(n == 0))) st = PMP_NO_PATH;  // OPEN exhausted (a_star.py:83)
        const lmask Mpop = Mact & ~Mpush & lm(n > 0);
        const bool pop = lb(Mpop);
        double Xf = lastf;
        uint32_t Xc = lastc, Xk = lastk;
        uint32_t Q = 0u;
        int Kd = 0;
        uint32_t ncm = rootc;  // the popped node (pop): its code, and the 3x3 round's loads
        int x = 0, y = 0;
        uint32_t nlin = 0u;
        uint32_t blk_w = 0u, blk_c = 0u;
        int blk_sh = 0;
        double gpar = 0.0;
        uint32_t ppar = 0u;  // THETA: Pc[pusher] (lane 13)
        Ld pld;
        // a push pair: the next two pending pushes, the first at an odd position (its sibling next);
        // heaps of >= 16 entries, so no cached parent (of positions <= n0 + 7) is a new leaf
        const uint32_t pend2 = pend & (pend - 1u);
        const lmask Mpair = kPair ? (Mpush & lm(pend2 != 0u) & lm((n & 1) != 0) & lm(n >= 16)) : 0ull;
        double X2f = 0.0;
        uint32_t X2c = 0u, X2k = 0u;
        if (push) {
            const int m = __ffs((int)pend) - 1;
            Xf = bpf(ifv, gb + m);
            Xc = bp(icm, gb + m);
            Xk = bp(ikk, gb + m);
            Q = (uint32_t)n + 1u;
            Kd = 31 - __clz((int)Q);
            if (kPair) {
                const int m2 = __ffs((int)pend2) - 1;  // (garbage lanes without a pair never use it)
                X2f = bpf(ifv, gb + (m2 & 7));
                X2c = bp(icm, gb + (m2 & 7));
                X2k = bp(ikk, gb + (m2 & 7));
            }
        }
        if (pop) {
            // ---- heappop (a_star.py:54), with the 3x3 round and the parent prefetch issued first
            npop++;
            n -= 1;
            n0 = n;
            const int ndir = cm_dir<HEUR>(ncm);
            x = ndir == 8 ? sx : gx - cm_dx<HEUR>(ncm);
            y = ndir == 8 ? sy : gy - cm_dy<HEUR>(ncm);
            const bool has_pusher = THETA ? ndir != 8 : ndir < 8;
            const int pm = ndir & 7;  // the pusher's motion
            nlin = (uint32_t)x * (uint32_t)H + (uint32_t)y;
            // every lane issues all three loads (lanes that need none read index 0): no branch per
            // lane class, so no load destination is zero-filled under another exec mask
            {
                const int cx = x + blk_dx, cy = y + blk_dy;
                const bool in_occ = gl < 9 && (unsigned)cx < (unsigned)W && (unsigned)cy < (unsigned)H;
                const uint32_t ci = in_occ ? (uint32_t)cx * (uint32_t)H + (uint32_t)cy : 0u;
                const uint32_t cti = in_occ ? cst_idx(cx, cy, tH) : 0u;
                const uint32_t pusher = !has_pusher ? 0u
                                        : THETA     ? gix(x - mot_x(pm), y - mot_y(pm))
                                                    : nlin - (uint32_t)(mot_x(pm) * H + mot_y(pm));
                const uint32_t gi = (!GZERO && gl == 12) ? pusher : 0u;
                const uint32_t ow = occ[ci >> 5];
                blk_c = cst[cti];
                gpar = GZERO ? 0.0 : G[gi];
                if (THETA) ppar = Pc[gl == 13 ? pusher : 0u];
                blk_sh = (int)(ci & 31u);
                blk_w = ow;
            }
            if (n > 0) pop_leaf<T2LDS>(hp, wk, n, gb, Q, Kd);
        }
        // the pushes will take positions n0, n0 + 1, ...: their parents, while all 8 share a depth
        Mpc = (Mpc & ~Mpop) | (Mpop & lm(n0 > 0) & lm(__clz(n0 + 1) == __clz(n0 + 8)));
        const int pp = (n0 + (gl & 7) - 1) >> 1;  // lanes 0..7: parent of position n0 + lane
        {
            const int pi = lb(Mpop & Mpc & kLanesLt8) ? pp : 0;
            pld.issue_off(hp, pi, soff(pi, pi >= hp.cap));
        }
        const lmask Mop = Mpush | (Mpop & lm(n > 0));
        double nf = 0.0;
        uint32_t nc = 0u, nk = 0u;
        int b = 0;
        b = path_op<T2LDS, HEUR>(hp, Mop, Mpop, Q, Kd, n, Xf, Xc, Xk, gl, gb, lastf, lastc, lastk, rootf, rootc, nf, nc,
                                 nk, cwL, Mpair, X2f, X2c, X2k);
        {
            double f8;
            uint32_t c8, k8;
            pld.get<HEUR>(f8, c8, k8);
            pf8 = pop ? f8 : pf8;
            pk8 = pop ? k8 : pk8;
        }
        // the cached parents (lanes 0..7: heap[parent(n0 + lane)]) after the operation: a position on
        // the path at a level the operation rewrote now holds that level's new content
        if (lb(Mop & Mpc)) {
            const int Lp = 31 - __clz(pp + 1);
            const bool onpath = lb(kLanesLt8 & lm(Lp <= Kd) & lm((int)(Q >> (Kd - Lp)) - 1 == pp) &
                                   ((Mpop & lm(Lp <= b)) | (~Mpop & lm(Lp >= b))));
            const int src = gb + (Lp < 16 ? Lp : 15);
            const double af = bpf(nf, src);
            const uint32_t ak = bp(nk, src);
            pf8 = onpath ? af : pf8;
            pk8 = onpath ? ak : pk8;
        }
        {
            const bool pr = lb(Mpair);
            pend = push ? (pr ? pend2 & (pend2 - 1u) : pend2) : pend;
            n += push ? (pr ? 2 : 1) : 0;
            npush += push ? (pr ? 2 : 1) : 0;
        }

        // ---- 3. the popped node: 3x3 masks (bit k = cell (x + k/3 - 1, y + k%3 - 1)), CLOSED test,
        //      goal test, getNeighbor (a_star.py:57-82)
        // lanes 0..8: the cell is in the grid
        const lmask Mblk = kLanesLt9 & lm((unsigned)(x + blk_dx) < (unsigned)W) & lm((unsigned)(y + blk_dy) < (unsigned)H);
        if (pop) {
            const uint32_t occ9 =
                (uint32_t)((kLanesLt9 & (~Mblk | lm(((blk_w >> blk_sh) & 1u) != 0u))) >> gb) & 0x1FFu;
            // a cell is CLOSED in this query when its byte's high nibble is the epoch and its low nibble
            // (motion + 1) is nonzero
            const uint32_t cls9 = (uint32_t)((Mblk & lm((blk_c >> 4) == ep) & lm((blk_c & 15u) != 0u)) >> gb) & 0x1FFu;
            const double gp = bcf<12>(gpar);
            if (!(cls9 & 16u)) {  // node.current not in CLOSED (a_star.py:57-58)
                const int ndir = cm_dir<HEUR>(ncm);
                double gnode = (GZERO || ndir == 8) ? 0.0 : gp + ((ndir & 1) ? kSqrt2 : 1.0);
                // THETA: the node's parent (cell, coordinates, g) and its expand-record code
                uint32_t par_lin = nlin;
                int px = x, py = y, ecode = ndir;
                double gp_g = 0.0;
                if (THETA && ndir != 8) {
                    const int pm = ndir & 7;
                    par_lin = nlin - (uint32_t)(mot_x(pm) * H + mot_y(pm));  // the pusher
                    gp_g = gp;
                    if (ndir >= 16) {  // path 2: node.g = parent.g + dist (theta_star.py:106-108)
                        par_lin = bc<13>(ppar);
                        const int qx = (int)(par_lin / (uint32_t)H), qy = (int)(par_lin - (uint32_t)qx * (uint32_t)H);
                        const double t = G[gl == 12 ? gix(qx, qy) : 0u];
                        gp_g = bcf<12>(t);
                    }
                    px = (int)(par_lin / (uint32_t)H);
                    py = (int)(par_lin - (uint32_t)px * (uint32_t)H);
                    gnode = gp_g + (ndir >= 16 ? __dsqrt_rn((double)((x - px) * (x - px) + (y - py) * (y - py)))
                                               : ((ndir & 1) ? kSqrt2 : 1.0));
                    if (THETA == 2 && !grid2d::los2d(occ, H, px, py, x, y)) {
                        // set vertex (lazy_theta_star.py:55-65): the first CLOSED, collision-free
                        // neighbour minimising its g + dist becomes the parent; g = inf if there is none
                        const bool cand = gl < 8 && (occ9 & nsb & 0xFFFFu) == 0u && (cls9 & (nsb >> 16)) != 0u;
                        const double gn = G[cand ? gix(x + mx, y + my) : 0u];
                        const double gc = gn + ((mo & 1) ? kSqrt2 : 1.0);
                        const uint32_t cmask = rbits(cand, gb) & 0xFFu;
                        double best = __longlong_as_double(0x7ff0000000000000ll);
                        int bm = -1;
                        for (int m = 0; m < 8; m++) {  // motion order, first minimum
                            const double c = bpf(gc, gb + m);
                            if (((cmask >> m) & 1u) && best > c) {
                                best = c;
                                bm = m;
                            }
                        }
                        gnode = best;
                        if (bm >= 0) {
                            gp_g = bpf(gn, gb + bm);
                            px = x + mot_x(bm);
                            py = y + mot_y(bm);
                            par_lin = (uint32_t)px * (uint32_t)H + (uint32_t)py;
                            ecode = 24 + bm;
                        } else {
                            ecode |= 32;
                        }
                    }
                }
                // CLOSED[node.current] = node (a_star.py:82)
                if (gl == 0) cst[cst_idx(x, y, tH)] = (uint8_t)((ep << 4) | (uint32_t)(THETA ? 1 : ndir + 1));
                if (!GZERO && gl == 1) G[gix(x, y)] = gnode;
                if (THETA && gl == 0) Pc[gix(x, y)] = par_lin;  // read back by this lane's extractPath
                if (mir8 && gl == 0) cst_m[cst_idx(x, y, tH)] = (uint8_t)((ep << 4) | (uint32_t)(ndir + 1));
                if (mir8 && !GZERO && gl == 1) G_m[gix(x, y)] = gnode;
                if (gl == 2 && expand_out && nexp < expand_cap)
                    expand_out[(size_t)q * expand_cap + nexp] =
                        THETA ? (nlin | ((uint32_t)ecode << 26)) : (nlin | ((uint32_t)ndir << 28));
                nexp++;
                if (x == gx && y == gy) {  // goal (a_star.py:61-64): extractPath, goal -> start
                    st = PMP_FOUND;
                    wave_sync_mem();
                    if (THETA && gl == 0) {  // via the CLOSED parents (any cell), hypot per hop
                        uint32_t li = nlin;
                        int cx = x, cy = y;
                        double cost = 0.0;
                        int len = 0;
                        uint32_t* pth = path_out + (size_t)q * path_cap;
                        for (;;) {
                            if (len < path_cap) pth[len] = li;
                            len++;
                            if (cx == sx && cy == sy) break;
                            const uint32_t pl = Pc[gix(cx, cy)];
                            const int qx = (int)(pl / (uint32_t)H), qy = (int)(pl - (uint32_t)qx * (uint32_t)H);
                            cost += __dsqrt_rn((double)((cx - qx) * (cx - qx) + (cy - qy) * (cy - qy)));
                            cx = qx;
                            cy = qy;
                            li = pl;
                        }
                        goal_cost = cost;
                        plen = len;
                    } else if (gl == 0) {
                        int cx = x, cy = y;
                        double cost = 0.0;
                        int len = 0;
                        uint32_t* pth = path_out + (size_t)q * path_cap;
                        for (;;) {
                            const uint32_t li = (uint32_t)cx * (uint32_t)H + (uint32_t)cy;
                            if (len < path_cap) pth[len] = li;
                            len++;
                            if (cx == sx && cy == sy) break;
                            const int d = (int)(cst[cst_idx(cx, cy, tH)] & 15u) - 1;
                            cost += (d & 1) ? kSqrt2 : 1.0;
                            cx -= mot_x(d);
                            cy -= mot_y(d);
                        }
                        goal_cost = cost;
                        plen = len;
                    }
                } else {
                    // getNeighbor in motion order; push the goal and stop (a_star.py:66-80)
                    const int ndx = gx - x - mx, ndy = gy - y - my;
                    const lmask Mnb = kLanesLt8 & lm((occ9 & nsb & 0xFFFFu) == 0u) & lm((cls9 & (nsb >> 16)) == 0u);
                    uint32_t vm = (uint32_t)(Mnb >> gb) & 0xFFu;
                    const uint32_t gm = (uint32_t)((Mnb & lm(ndx == 0) & lm(ndy == 0)) >> gb) & 0xFFu;
                    if (gm) vm &= (gm << 1) - 1u;
                    double ig = gnode + (GZERO ? 0.0 : ((mo & 1) ? kSqrt2 : 1.0));
                    int icode = mo;
                    if (THETA && ndir != 8) {
                        // updateVertex(CLOSED[node.parent], node_n) (theta_star.py:96-108; lazy_theta_star.py:
                        // 103-114 without the line of sight): path 2 when parent.g + dist <= node_n.g
                        const int nxl = x + mx, nyl = y + my;
                        const double g2 = gp_g + __dsqrt_rn((double)((px - nxl) * (px - nxl) + (py - nyl) * (py - nyl)));
                        if (gl < 8 && ((vm >> mo) & 1u) && g2 <= ig &&
                            (THETA == 2 || grid2d::los2d(occ, H, nxl, nyl, px, py))) {
                            ig = g2;
                            icode = 16 + mo;
                        }
                    }
                    icm = pack_cm<HEUR>(ndx, ndy, icode);
                    ikk = hkey<HEUR>(icm);
                    ifv = ig + h_of_key<HEUR>(ikk);
                    if (n + __popc(vm) > heap_cap) st = PMP_CAP_OVERFLOW;  // a push would find n >= heap_cap
                    else pend = vm;
                }
            }
        }
        if (n > maxn) maxn = n;

        // ---- the groups whose query ended: results, then a new query next step
        const lmask Mend = lm(st >= 0);
        Mneed |= Mend;
        if (lb(Mend)) {
            if (gl == 0) {
                int s = st;
                if (s == PMP_FOUND && plen > path_cap) s = PMP_PATH_OVERFLOW;
                status_out[q] = s;
                cost_out[q] = st == PMP_FOUND ? goal_cost : 0.0;
                path_len_out[q] = st == PMP_FOUND ? plen : 0;
                nexp_out[q] = nexp;
                if (counters) {
                    counters[4 * q + 0] = (int64_t)npush;
                    counters[4 * q + 1] = (int64_t)npop;
                    counters[4 * q + 2] = nexp;
                    counters[4 * q + 3] = maxn;
                }
            }
            pend = 0u;
        }
    }
    if (gl == 0) epoch_all[slot] = ep;
    span_end(span);
}

size_t mq_cst_bytes(int W, int H) { return (cst_tiled_bytes(W, H) + 255) & ~(size_t)255; }

}  // namespace

// Per-slot query state shared by the multi-query and the single-query engines: cell-state bytes
// ((epoch << 4) | motion + 1), G, and the slot's epoch.  Any launch may use any slot under the epoch
// protocol; a new layout (more slots, another grid size) resets every epoch, so each slot clears its
// cell states at its first query.
int pmp_astar2d_slot_scratch(pmp_ctx* ctx, hipStream_t s, size_t slots, int W, int H, uint8_t** cst, size_t* cst_bytes,
                             double** G, uint32_t** ep)
{
    const size_t cb = mq_cst_bytes(W, H);
    const size_t gsc = g_slot_cells(W, H);
    const size_t ms = (kMirror & 8) ? slots + slots / 2 + 1 : slots;  // kMirror: the even slots' mirrors
    *cst = (uint8_t*)pmp_scratch(ctx, SCR_MQ_CST, ms * cb + 16);
    *G = (double*)pmp_scratch(ctx, SCR_MQ_G, ms * gsc * 8 + 16);
    const bool fresh_epochs = ctx->cap[SCR_MQ_EPOCH] < slots * 4 || ctx->astar_mq_epoch_slots < slots ||
                              ctx->astar_mq_cst_bytes != cb;
    *ep = (uint32_t*)pmp_scratch(ctx, SCR_MQ_EPOCH, slots * 4 + 16);
    if (!*cst || !*G || !*ep) return PMP_ENOMEM;
    if (fresh_epochs) {
        PMP_HIP_CHECK(ctx, hipMemsetAsync(*ep, 0, slots * 4 + 16, s));
        ctx->astar_mq_epoch_slots = slots;
        ctx->astar_mq_cst_bytes = cb;
    }
    *cst_bytes = cb;
    return PMP_OK;
}

// The multi-query engine's launch (called by pmp_graph2d_batch for A* / Dijkstra / GBFS when the
// context's heap capacity fits kMqCap).  ctx->astar_workers = group slots (queries in flight) of
// one launch; the LDS share per group comes from the residency (groups per CU over all launches in
// flight).
int pmp_astar2d_mq_launch(pmp_ctx* ctx, hipStream_t s, int algo, const uint32_t* occ_bits, int W, int H, int heuristic,
                          const int32_t* start_xy, const int32_t* goal_xy, const int32_t* order, int nq, double* cost,
                          int32_t* path_len, uint32_t* path, int path_cap, int32_t* n_expanded, uint32_t* expand,
                          int expand_cap, int64_t* counters, int32_t* status, int* queue)
{
    int groups = ctx->astar_workers < nq ? ctx->astar_workers : nq;
    const bool t2lds = ctx->astar_mq_t2lds != 0;
    const int bits_b = t2lds ? kBits01 + kT2LBytes : kBits01;
    const int cap_max = t2lds ? kMqCapT2L : kMqCap;
    const int heap_cap = ctx->astar_heap_cap < cap_max ? ctx->astar_heap_cap : cap_max;
    const int theta = algo == PMP_ALGO_THETA ? 1 : (algo == PMP_ALGO_LAZY_THETA ? 2 : 0);
    if (theta) {
        // the reservation's fit (astar2d_reserve_impl) counts cell state, G, spill and bits per slot;
        // Theta* adds a W*H*4-byte CLOSED-parent array per slot: fewer groups (the persistent queue
        // serves every query) instead of growing past the budget
        const size_t per_slot = (size_t)W * H + g_slot_cells(W, H) * 12 + (size_t)cap_max * 16 + 4096 + 256;
        const size_t fit = (kScratchBudgetMq / per_slot) & ~(size_t)3;
        if (fit < 4) return pmp_set_err(ctx, PMP_ENOMEM, "ThetaStar: one wave's slots exceed the scratch budget");
        if ((size_t)groups > fit) groups = (int)fit;
    }
    // lone: fewer queries than CUs -- one query per wave, in group 0, with the CU's whole LDS as its
    // heap share (the drop-in single query: latency, not throughput)
    const bool lone = nq <= kMqLoneMax;
    const int waves = lone ? nq : (groups + 3) / 4;
    int lds_cap = ctx->astar_lds_cap;
    if (lone) {
        lds_cap = ((160 * 1024 - 256 - bits_b) / kEntLds) & ~15;
        if (lds_cap > heap_cap) lds_cap = (heap_cap + 15) & ~15;
    }
    const int region = bits_b + kEntLds * lds_cap;
    int spill_n = ((heap_cap > lds_cap ? heap_cap - lds_cap : 1) + kSpillShift + 1) & ~1;
    if (kBlocks) {  // 16-B units of the group's blocks: bands of two levels from L0 to the deepest level
        const int L0 = 31 - __builtin_clz((unsigned)lds_cap + 1u);
        const int Lmax = 31 - __builtin_clz((unsigned)(heap_cap > 1 ? heap_cap : 2));
        const int B = Lmax >= L0 ? (Lmax - L0) / 2 + 1 : 1;
        const size_t blocks = ((size_t)1 << (L0 - 1)) * ((((size_t)1 << (2 * B)) - 1) / 3);
        spill_n = (int)(blocks * 8);
    }
    const size_t slots = (size_t)waves * 4;
    uint4* spill = (uint4*)pmp_scratch(ctx, SCR_MQ_SPILL, (kMirror & 7 ? 2 : 1) * slots * (size_t)spill_n * 16 + 16);
    uint32_t* t2 = (uint32_t*)pmp_scratch(ctx, SCR_MQ_T2, slots * kT2Words * 4 + 16);
    if (!spill || !t2) return PMP_ENOMEM;
    uint32_t* Pc = nullptr;  // Theta*: the CLOSED parent cell of every cell, per slot
    if (theta) {
        Pc = (uint32_t*)pmp_scratch(ctx, SCR_MQ_PC, slots * g_slot_cells(W, H) * 4 + 16);
        if (!Pc) return PMP_ENOMEM;
    }
    uint8_t* cstp;
    size_t cst_bytes;
    double* G;
    uint32_t* ep;
    {
        const int rc = pmp_astar2d_slot_scratch(ctx, s, slots, W, H, &cstp, &cst_bytes, &G, &ep);
        if (rc) return rc;
    }
    const size_t lds = (size_t)region * (lone ? 1 : 4);
    const int prio = order ? ctx->astar_prio_n : 0;
#define MQ_LAUNCH_T(HE, GZ, T2, TH)                                                                                 \
    hipLaunchKernelGGL((astar2d_mqu_kernel<HE, GZ, T2, TH>), dim3(waves), dim3(64), lds, s, occ_bits, W, H, start_xy, \
                       goal_xy, order, nq, cost, path_len, path, path_cap, n_expanded, expand, expand_cap, counters, \
                       status, queue, spill, spill_n, heap_cap, lds_cap, region, cstp, cst_bytes, G, t2, ep, prio,   \
                       lone ? 1 : 0, ctx->span, Pc)
#define MQ_LAUNCH(HE, GZ, T2) MQ_LAUNCH_T(HE, GZ, T2, 0)
    const int he = algo == PMP_ALGO_DIJKSTRA ? 2 : heuristic;
    const bool gz = algo == PMP_ALGO_GBFS;
    constexpr int TL = kThetaLayout;
    if (theta) {
        if (t2lds) {
            if (theta == 1) { if (he == 1) MQ_LAUNCH_T(TL | 1, false, true, 1); else MQ_LAUNCH_T(TL, false, true, 1); }
            else { if (he == 1) MQ_LAUNCH_T(TL | 1, false, true, 2); else MQ_LAUNCH_T(TL, false, true, 2); }
        } else {
            if (theta == 1) { if (he == 1) MQ_LAUNCH_T(TL | 1, false, false, 1); else MQ_LAUNCH_T(TL, false, false, 1); }
            else { if (he == 1) MQ_LAUNCH_T(TL | 1, false, false, 2); else MQ_LAUNCH_T(TL, false, false, 2); }
        }
    } else if (t2lds) {
        if (gz) { if (he == 1) MQ_LAUNCH(1, true, true); else MQ_LAUNCH(0, true, true); }
        else if (he == 2) MQ_LAUNCH(2, false, true);
        else if (he == 1) MQ_LAUNCH(1, false, true);
        else MQ_LAUNCH(0, false, true);
    } else {
        if (gz) { if (he == 1) MQ_LAUNCH(1, true, false); else MQ_LAUNCH(0, true, false); }
        else if (he == 2) MQ_LAUNCH(2, false, false);
        else if (he == 1) MQ_LAUNCH(1, false, false);
        else MQ_LAUNCH(0, false, false);
    }
#undef MQ_LAUNCH
#undef MQ_LAUNCH_T
    PMP_HIP_CHECK(ctx, hipGetLastError());
    return PMP_OK;
}

// LDS heap positions per group for `per_cu` groups resident per CU (each CU's 160 KiB shared)
int pmp_astar2d_mq_lds_cap(int per_cu, bool t2lds)
{
    const int bits_b = t2lds ? kBits01 + kT2LBytes : kBits01;
    // a workgroup is one wave = 4 groups, and may hold at most the CU's 160 KiB
    int bytes = (160 * 1024) / (per_cu < 4 ? 4 : per_cu) - 160 - bits_b;
    int cap = (bytes / kEntLds) & ~15;
    if (cap > kMqCap) cap = kMqCap & ~15;
    return cap;
}
int pmp_astar2d_mq_cap(bool t2lds) { return t2lds ? kMqCapT2L : kMqCap; }
