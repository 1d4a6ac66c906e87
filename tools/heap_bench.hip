// Dev microbenchmark: cycles per pop / push of the heap16.h engine in isolation (LDS-resident
// heap, one wave per block, 4 blocks per CU as in the 3D A* kernel).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../python_motion_planning_amd/csrc heap_bench.hip -o heap_bench
#include <cstdio>
#include <vector>

#include "heap16.h"

using heap16::Ent;

struct KeyT {
    __device__ __forceinline__ void derive(Ent& e) const { e.f = e.g; e.hk = e.b; }
    static __device__ __forceinline__ bool lt(const Ent& x, const Ent& y)
    {
        return (x.f < y.f) | ((x.f == y.f) & ((x.hk < y.hk) | ((x.hk == y.hk) & (x.a < y.a))));
    }
};

// heap16::pop with phase stamps: [0] last load, [1] child loads+derive+ballots, [2] walk, [3] stores
template <class K>
__device__ void pop_stamped(const heap16::Heap& hp, const K& key, int n, Ent& root, int lane, int jl, int ol,
                            unsigned long long* ph)
{
    using namespace heap16;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    n = uni(n);
    Ent last;
    load<false>(hp, n, last);
    last.g = rl_f64(last.g, 0);
    last.a = rl_u32(last.a, 0);
    last.b = rl_u32(last.b, 0);
    key.derive(last);
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    ph[0] += t1 - t0;
    int hole = 0;
    bool first = true;
    for (;;) {
        t0 = __builtin_amdgcn_s_memtime();
        const int li = ((hole + 1) << jl) - 1 + 2 * ol;
        const bool vl = (lane < 63) & (li < n);
        const bool vr = (lane < 63) & (li + 1 < n);
        Ent L, R;
        load<false>(hp, vl ? li : 0, L);
        load<false>(hp, vr ? li + 1 : 0, R);
        key.derive(L);
        key.derive(R);
        const uint64_t dmask = ballot(vr & K::lt(R, L));
        const uint64_t mlmask = ballot(vl & K::lt(L, last));
        const uint64_t mrmask = ballot(vr & K::lt(R, last));
        t1 = __builtin_amdgcn_s_memtime();
        int cur = uni(hole), oc = 0;
        uint64_t mover = 0, movr = 0;
        uint32_t go = 1u;
#pragma unroll
        for (int lv = 1; lv <= 6; lv++) {
            const int c = 2 * cur + 1;
            const int pl = (1 << (lv - 1)) - 1 + oc;
            const uint32_t r = (uint32_t)(dmask >> pl) & 1u;
            const uint64_t mm = r ? mrmask : mlmask;
            go = go & (uint32_t)(c < n) & ((uint32_t)(mm >> pl) & 1u);
            const uint64_t bit = (uint64_t)go << pl;
            mover |= bit;
            movr |= (uint64_t)(go & r) << pl;
            cur = go ? c + (int)r : cur;
            oc = go ? 2 * oc + (int)r : oc;
        }
        const unsigned long long t2 = __builtin_amdgcn_s_memtime();
        if ((mover >> lane) & 1ull) {
            const bool rr = (movr >> lane) & 1ull;
            store<false>(hp, ((rr ? li + 1 : li) - 1) >> 1, rr ? R : L);
        }
        if (first && (mover & 1ull)) root = rl_ent((movr & 1ull) ? R : L, 0);
        first = false;
        hole = cur;
        const unsigned long long t3 = __builtin_amdgcn_s_memtime();
        ph[1] += t1 - t0;
        ph[2] += t2 - t1;
        ph[3] += t3 - t2;
        ph[4] += 1;
        if (!go) break;
        wsync();
    }
    if (lane == 0) store<false>(hp, hole, last);
    if (hole == 0) root = last;
    wsync();
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u4;
__device__ __forceinline__ void ldA(const lds_u4* H, int p, Ent& e)
{
    const u32x4 v = H[p];
    e.g = __hiloint2double((int)v.y, (int)v.x);
    e.a = v.z;
    e.b = v.w;
}
__device__ __forceinline__ void stA(lds_u4* H, int p, const Ent& e)
{
    const uint64_t bits = (uint64_t)__double_as_longlong(e.g);
    u32x4 v;
    v.x = (uint32_t)bits; v.y = (uint32_t)(bits >> 32); v.z = e.a; v.w = e.b;
    H[p] = v;
}

// AoS heap (one 16 B record per entry, one ds_read_b128 per child)
template <class K>
__device__ void popA(lds_u4* H, const K& key, int n, Ent& root, int lane, int jl, int ol)
{
    using namespace heap16;
    n = uni(n);
    Ent last;
    ldA(H, n, last);
    last.g = rl_f64(last.g, 0);
    last.a = rl_u32(last.a, 0);
    last.b = rl_u32(last.b, 0);
    key.derive(last);
    int hole = 0;
    bool first = true;
    for (;;) {
        const int li = ((hole + 1) << jl) - 1 + 2 * ol;
        const bool vl = (lane < 63) & (li < n);
        const bool vr = (lane < 63) & (li + 1 < n);
        Ent L, R;
        ldA(H, vl ? li : 0, L);
        ldA(H, vr ? li + 1 : 0, R);
        key.derive(L);
        key.derive(R);
        const uint64_t dmask = ballot(vr & K::lt(R, L));
        const uint64_t mlmask = ballot(vl & K::lt(L, last));
        const uint64_t mrmask = ballot(vr & K::lt(R, last));
        int cur = uni(hole), oc = 0;
        uint64_t mover = 0, movr = 0;
        uint32_t go = 1u;
#pragma unroll
        for (int lv = 1; lv <= 6; lv++) {
            const int c = 2 * cur + 1;
            const int pl = (1 << (lv - 1)) - 1 + oc;
            const uint32_t r = (uint32_t)(dmask >> pl) & 1u;
            const uint64_t mm = r ? mrmask : mlmask;
            go = go & (uint32_t)(c < n) & ((uint32_t)(mm >> pl) & 1u);
            const uint64_t bit = (uint64_t)go << pl;
            mover |= bit;
            movr |= (uint64_t)(go & r) << pl;
            cur = go ? c + (int)r : cur;
            oc = go ? 2 * oc + (int)r : oc;
        }
        if ((mover >> lane) & 1ull) {
            const bool rr = (movr >> lane) & 1ull;
            stA(H, ((rr ? li + 1 : li) - 1) >> 1, rr ? R : L);
        }
        if (first && (mover & 1ull)) root = rl_ent((movr & 1ull) ? R : L, 0);
        first = false;
        hole = cur;
        if (!go) break;
        wsync();
    }
    if (lane == 0) stA(H, hole, last);
    if (hole == 0) root = last;
    wsync();
}

template <class K>
__device__ void pushA(lds_u4* H, const K& key, int n, const Ent& it, Ent& root, int lane)
{
    using namespace heap16;
    n = uni(n);
    const int np1 = n + 1;
    const int depth = 31 - __clz(np1);
    const bool valid = lane < depth;
    const int apos = valid ? (np1 >> (lane + 1)) - 1 : 0;
    Ent a;
    ldA(H, apos, a);
    key.derive(a);
    const int t = __popcll(ballot(valid & K::lt(it, a)));
    if (lane < t) stA(H, (np1 >> lane) - 1, a);
    const int ipos = (np1 >> t) - 1;
    if (lane == 0) stA(H, ipos, it);
    if (ipos == 0) root = it;
    wsync();
}

__global__ __launch_bounds__(64) void benchA(int n0, int iters, unsigned long long* out)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    lds_u4* H = (lds_u4*)smem;
    const int lane = lane_id();
    int jl, ol;
    heap16::pop_lane_consts(lane, jl, ol);
    const KeyT key;
    uint32_t rng = 12345u + blockIdx.x * 7919u;
    auto nextf = [&]() {
        rng = rng * 1664525u + 1013904223u;
        return (double)(rng >> 8) * (1.0 / 16777216.0);
    };
    Ent root;
    root.g = 0.0; root.a = 0; root.b = 0;
    key.derive(root);
    if (lane == 0) stA(H, 0, root);
    heap16::wsync();
    int n = 1;
    uint32_t seq = 1;
    double base = 0.0;
    for (int i = 1; i < n0; i++) {
        Ent it;
        it.g = base + nextf(); it.a = seq++; it.b = 0;
        key.derive(it);
        pushA<KeyT>(H, key, n, it, root, lane);
        n++;
    }
    unsigned long long c_pop = 0, c_push = 0;
    for (int i = 0; i < iters; i++) {
        base = root.g;
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        n -= 1;
        popA<KeyT>(H, key, n, root, lane, jl, ol);
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        Ent it;
        it.g = base + nextf(); it.a = seq++; it.b = 0;
        key.derive(it);
        pushA<KeyT>(H, key, n, it, root, lane);
        n++;
        const unsigned long long t2 = __builtin_amdgcn_s_memtime();
        c_pop += t1 - t0;
        c_push += t2 - t1;
    }
    if (lane == 0) { out[2 * blockIdx.x] = c_pop; out[2 * blockIdx.x + 1] = c_push; }
}

__global__ __launch_bounds__(64) void bench_phases(int n0, int iters, int lds_cap, unsigned long long* out)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = lane_id();
    const heap16::Heap hp = heap16::make_heap(smem, lds_cap, nullptr, 0);
    int jl, ol;
    heap16::pop_lane_consts(lane, jl, ol);
    const KeyT key;
    uint32_t rng = 12345u + blockIdx.x * 7919u;
    auto nextf = [&]() {
        rng = rng * 1664525u + 1013904223u;
        return (double)(rng >> 8) * (1.0 / 16777216.0);
    };
    Ent root;
    root.g = 0.0; root.a = 0; root.b = 0;
    key.derive(root);
    if (lane == 0) heap16::store<false>(hp, 0, root);
    heap16::wsync();
    int n = 1;
    uint32_t seq = 1;
    double base = 0.0;
    for (int i = 1; i < n0; i++) {
        Ent it;
        it.g = base + nextf(); it.a = seq++; it.b = 0;
        key.derive(it);
        heap16::push<KeyT, false>(hp, key, n, it, root, lane);
        n++;
    }
    unsigned long long ph[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < iters; i++) {
        base = root.g;
        n -= 1;
        pop_stamped<KeyT>(hp, key, n, root, lane, jl, ol, ph);
        Ent it;
        it.g = base + nextf(); it.a = seq++; it.b = 0;
        key.derive(it);
        heap16::push<KeyT, false>(hp, key, n, it, root, lane);
        n++;
    }
    if (lane == 0)
        for (int k = 0; k < 5; k++) out[5 * blockIdx.x + k] = ph[k];
}

__global__ __launch_bounds__(64) void bench(int n0, int iters, int lds_cap, unsigned long long* out)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = lane_id();
    const heap16::Heap hp = heap16::make_heap(smem, lds_cap, nullptr, 0);
    int jl, ol;
    heap16::pop_lane_consts(lane, jl, ol);
    const KeyT key;
    uint32_t rng = 12345u + blockIdx.x * 7919u;
    auto nextf = [&]() {
        rng = rng * 1664525u + 1013904223u;
        return (double)(rng >> 8) * (1.0 / 16777216.0);
    };
    Ent root;
    root.g = 0.0; root.a = 0; root.b = 0;
    key.derive(root);
    if (lane == 0) heap16::store<false>(hp, 0, root);
    heap16::wsync();
    int n = 1;
    uint32_t seq = 1;
    double base = 0.0;
    for (int i = 1; i < n0; i++) {
        Ent it;
        it.g = base + nextf();
        it.a = seq++;
        it.b = 0;
        key.derive(it);
        heap16::push<KeyT, false>(hp, key, n, it, root, lane);
        n++;
    }
    unsigned long long c_pop = 0, c_push = 0;
    for (int i = 0; i < iters; i++) {
        base = root.g;
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        n -= 1;
        heap16::pop<KeyT, false>(hp, key, n, root, lane, jl, ol);
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        Ent it;
        it.g = base + nextf();
        it.a = seq++;
        it.b = 0;
        key.derive(it);
        heap16::push<KeyT, false>(hp, key, n, it, root, lane);
        n++;
        const unsigned long long t2 = __builtin_amdgcn_s_memtime();
        c_pop += t1 - t0;
        c_push += t2 - t1;
    }
    if (lane == 0) {
        out[2 * blockIdx.x] = c_pop;
        out[2 * blockIdx.x + 1] = c_push;
    }
}

int main()
{
    const int blocks = 1024, iters = 20000;
    for (int n0 : {100, 1000, 2000}) {
        const int lds_cap = 2288;
        unsigned long long* d;
        hipMalloc(&d, sizeof(unsigned long long) * 2 * blocks);
        hipLaunchKernelGGL(bench, dim3(blocks), dim3(64), lds_cap * 16, 0, n0, iters, lds_cap, d);
        std::vector<unsigned long long> h(2 * blocks);
        hipMemcpy(h.data(), d, sizeof(unsigned long long) * 2 * blocks, hipMemcpyDeviceToHost);
        double sp = 0, su = 0;
        for (int b = 0; b < blocks; b++) { sp += h[2 * b]; su += h[2 * b + 1]; }
        printf("heap %5d entries: pop %.0f cycles, push %.0f cycles (1024 waves, 4 per CU)\n", n0,
               sp / blocks / iters, su / blocks / iters);
        hipFree(d);
    }
    for (int n0 : {100, 1000, 2000}) {
        unsigned long long* d;
        hipMalloc(&d, sizeof(unsigned long long) * 2 * blocks);
        hipLaunchKernelGGL(benchA, dim3(blocks), dim3(64), 2288 * 16, 0, n0, iters, d);
        std::vector<unsigned long long> h(2 * blocks);
        hipMemcpy(h.data(), d, sizeof(unsigned long long) * 2 * blocks, hipMemcpyDeviceToHost);
        double sp = 0, su = 0;
        for (int b = 0; b < blocks; b++) { sp += h[2 * b]; su += h[2 * b + 1]; }
        printf("AoS heap %5d entries: pop %.0f cycles, push %.0f cycles\n", n0, sp / blocks / iters, su / blocks / iters);
        hipFree(d);
    }
    {
        const int lds_cap = 2288, n0 = 1000;
        unsigned long long* d;
        hipMalloc(&d, sizeof(unsigned long long) * 5 * blocks);
        hipLaunchKernelGGL(bench_phases, dim3(blocks), dim3(64), lds_cap * 16, 0, n0, iters, lds_cap, d);
        std::vector<unsigned long long> h(5 * blocks);
        hipMemcpy(h.data(), d, sizeof(unsigned long long) * 5 * blocks, hipMemcpyDeviceToHost);
        double t[5] = {0, 0, 0, 0, 0};
        for (int b = 0; b < blocks; b++)
            for (int k = 0; k < 5; k++) t[k] += h[5 * b + k];
        printf("phases (heap %d): last-load %.0f per pop; per round: loads+ballots %.0f, walk %.0f, stores %.0f; "
               "rounds/pop %.2f\n", n0, t[0] / blocks / iters, t[1] / t[4], t[2] / t[4], t[3] / t[4], t[4] / blocks / iters);
    }
    return 0;
}
