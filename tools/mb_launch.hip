// mb_launch.hip - micro-benchmark (development tool, not product code): what a
// dependent kernel launch costs OUTSIDE its workgroups, one resource at a time.
//
// Every variant is a HIP graph of N dependent launches of 256 (or 512)
// workgroups of 256 threads (the sub-talker GEMVs' geometry).  Reported per
// variant:
//   us/kernel  graph replay time / N (HIP events)              = the wall per launch
//   span       median over launches of (last workgroup's end - first
//              workgroup's start), s_memrealtime (100 MHz) stamps
//   gap        median of (first start of launch i+1 - last end of launch i)
//   ramp       median of (last workgroup's start - first's)
// Running the binary under `rocprofv3 --kernel-trace --stats` gives each
// variant's rocprof average duration beside them (kernel names below).
//
// Variants (each changes ONE thing against `x4k`):
//   empty        no arguments, no body
//   stamp        the stamps alone (one int kernarg)
//   x4k          reads the previous launch's 4 KB output (float4 per thread),
//                wave + LDS sum, writes 4 floats per workgroup (all-to-all edge)
//   x4k_big      the same through a 256-B by-value struct kernarg (GemvArgs-like)
//   x4k_vgpr     + 256 VGPRs allocated (an asm clobber of v255)
//   x4k_lds      + 64 KB of dynamic LDS
//   x4k_code     + 24 KB of straight-line code executed once (I-cache misses)
//   x4k_code4    four such kernels in rotation (96 KB of code between reuses)
//   x4k_loop     the same instruction count as a loop over a 96-B body
//   x4k_resid    + y[r] += v epilogue (a dependent read-modify-write of the output)
//   x32k / x64k  every workgroup reads the previous launch's whole 32 / 64 KB
//                output (the batch GEMVs' x of 8 rows); _rep8: the output in 8
//                copies, each XCD's workgroups reading their own
//   gemv_gu      the sub-talker gate|up shape (6144 x 1024 bf16, Infinity-Cache
//                resident), whole weight slice in flight before x (k_gemvw-like)
//
//   hipcc -O3 --offload-arch=gfx950 tools/mb_launch.hip -o tools/mb_launch && tools/mb_launch
//   (add -mllvm -amdgpu-kernarg-preload-count=16 for the preloaded-kernarg build)
#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <string.h>

#include <algorithm>
#include <vector>

// every HIP call announces itself on stderr first (unbuffered): a fault inside
// the runtime (the SIGSEGV under rocprofv3 --kernel-trace in round 4) then
// names the call it happened in
static int g_trace = 1;
#define CK(x) do { if (g_trace) fprintf(stderr, "[mb_launch] %s:%d %s\n", __func__, __LINE__, #x); \
                    hipError_t e = (x); if (e != hipSuccess) { printf("%s failed: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr int NL = 200, MAXG = 512;
__device__ unsigned long long g_st[NL][MAXG][2];

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ void stamp_end(int i, unsigned long long t0) {
    const unsigned long long t1 = now();
    if (threadIdx.x == 0) { g_st[i][blockIdx.x][0] = t0; g_st[i][blockIdx.x][1] = t1; }
}
__device__ __forceinline__ float wsum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// 4 KB in -> 4 floats per workgroup out (grid 256: 1024 floats = the next 4 KB)
__device__ __forceinline__ float x4k_body(const float *in, float *red) {
    const float4 v = reinterpret_cast<const float4 *>(in)[threadIdx.x];
    const float s = wsum(v.x + v.y + v.z + v.w);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    return red[threadIdx.x & 3];
}

__global__ void k_empty() {}
__global__ __launch_bounds__(256) void k_stamp(int i) { const auto t0 = now(); stamp_end(i, t0); }
__global__ __launch_bounds__(256) void k_x4k(int i, const float *in, float *out) {
    const auto t0 = now();
    __shared__ float red[4];
    const float s = x4k_body(in, red);
    if (threadIdx.x < 4) out[blockIdx.x * 4 + threadIdx.x] = s * 0.25f;
    stamp_end(i, t0);
}
struct Big { int i; int pad0; const float *in; float *out; float pad[58]; };   // 256 B
__global__ __launch_bounds__(256) void k_x4k_big(Big a) {
    const auto t0 = now();
    __shared__ float red[4];
    const float s = x4k_body(a.in, red);
    if (threadIdx.x < 4) a.out[blockIdx.x * 4 + threadIdx.x] = s * 0.25f + a.pad[threadIdx.x & 31];
    stamp_end(a.i, t0);
}
// the kernarg-size sweep (--kernarg-sweep): the x4k body through a by-value
// struct of B bytes
template <int B>
struct KB { int i; int pad0; const float *in; float *out; float pad[(B - 24) / 4]; };
template <int B>
__global__ __launch_bounds__(256) void k_x4k_kb(KB<B> a) {
    static_assert(sizeof(KB<B>) == B, "kernarg size");
    const auto t0 = now();
    float s = wsum(a.in[threadIdx.x + 256 * 0]);
    if ((threadIdx.x & 63) == 0) a.out[blockIdx.x * 4 + (threadIdx.x >> 6)] = s + a.pad[0];
    stamp_end(a.i, t0);
}
__global__ __launch_bounds__(256) void k_x4k_vgpr(int i, const float *in, float *out) {
    const auto t0 = now();
    __shared__ float red[4];
    const float s = x4k_body(in, red);
    asm volatile("; force 256 VGPRs" ::: "v255");
    if (threadIdx.x < 4) out[blockIdx.x * 4 + threadIdx.x] = s * 0.25f;
    stamp_end(i, t0);
}
__global__ __launch_bounds__(256) void k_x4k_lds(int i, const float *in, float *out) {
    const auto t0 = now();
    extern __shared__ float dyn[];
    const float s = x4k_body(in, dyn);
    if (threadIdx.x < 4) out[blockIdx.x * 4 + threadIdx.x] = s * 0.25f;
    stamp_end(i, t0);
}
#define A4 "v_add_f32 %0, %0, %1\n"
#define A16 A4 A4 A4 A4
#define A64 A16 A16 A16 A16
#define A256 A64 A64 A64 A64
template <int V>
__global__ __launch_bounds__(256) void k_x4k_code(int i, const float *in, float *out) {
    const auto t0 = now();
    __shared__ float red[4];
    float s = x4k_body(in, red);
    float a = s;
    // 24 x 256 v_add_f32_e32 (4 B each) = 24 KB of straight-line code
    asm volatile(A256 A256 A256 A256 A256 A256 A256 A256 A256 A256 A256 A256
                 A256 A256 A256 A256 A256 A256 A256 A256 A256 A256 A256 A256 : "+v"(a) : "v"(s));
    if (threadIdx.x < 4) out[blockIdx.x * 4 + threadIdx.x] = a + (float)V;
    stamp_end(i, t0);
}
__global__ __launch_bounds__(256) void k_x4k_loop(int i, const float *in, float *out) {
    const auto t0 = now();
    __shared__ float red[4];
    float s = x4k_body(in, red);
    float a = s;
    for (int k = 0; k < 256; ++k) asm volatile(A16 A4 A4 : "+v"(a) : "v"(s));   // 256 x 24 adds
    if (threadIdx.x < 4) out[blockIdx.x * 4 + threadIdx.x] = a;
    stamp_end(i, t0);
}
__global__ __launch_bounds__(256) void k_x4k_resid(int i, const float *in, float *out) {
    const auto t0 = now();
    __shared__ float red[4];
    const float s = x4k_body(in, red);
    if (threadIdx.x < 4) out[blockIdx.x * 4 + threadIdx.x] += s * 0.25f;
    stamp_end(i, t0);
}
// The batch GEMVs' x fetch: every workgroup reads the previous launch's
// whole KB-KB output (KB = 32 / 64: the sub-talker / talker x of 8 batch
// rows) and writes its KB floats of the next; REP = 1: the output is stored
// in 8 copies and workgroup b reads the copy of its XCD, (b + 7) % 8
// (profiles/r05a_mb_l2pf_xcc.txt), so the 8 XCDs' misses go to 8 different
// sets of lines instead of all to one
template <int KB, int REP>
__global__ __launch_bounds__(256) void k_xbig(int i, const float *in, float *out) {
    const auto t0 = now();
    __shared__ float red[4];
    constexpr int N = KB * 256, J = N / 1024;
    const int c = REP ? (blockIdx.x + 7) % 8 : 0;
    const float *src = in + (size_t)c * N;
    float4 v[J];
#pragma unroll
    for (int j = 0; j < J; ++j) v[j] = reinterpret_cast<const float4 *>(src)[threadIdx.x + 256 * j];
    float a = 0.f;
#pragma unroll
    for (int j = 0; j < J; ++j) a += v[j].x + v[j].y + v[j].z + v[j].w;
    const float sw = wsum(a);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sw;
    __syncthreads();
    const float s = (red[0] + red[1] + red[2] + red[3]) * 1e-3f;
    if (threadIdx.x < KB) {
#pragma unroll
        for (int cc = 0; cc < (REP ? 8 : 1); ++cc) out[(size_t)cc * N + blockIdx.x * KB + threadIdx.x] = s;
    }
    stamp_end(i, t0);
}

// gate|up-like: grid 256, 24 rows per workgroup (RW 6), C = 1024 (NV 2)
__global__ __launch_bounds__(256) void k_gemv_gu(int i, const uint16_t *W, const float *in, float *out) {
    const auto t0 = now();
    __shared__ __attribute__((aligned(16))) float xs[1024];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const float4 xv = reinterpret_cast<const float4 *>(in)[threadIdx.x];
    v4u wv[6][2];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int k = 0; k < 2; ++k)
            wv[r][k] = reinterpret_cast<const v4u *>(W + (size_t)(blockIdx.x * 24 + w + 4 * r) * 1024)[lane + 64 * k];
    reinterpret_cast<float4 *>(xs)[threadIdx.x] = xv;
    __syncthreads();
    float acc[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const float *x = xs + 8 * (lane + 64 * k);
            const v4u q = wv[r][k];
            s = fmaf(__uint_as_float(q.x << 16), x[0], s); s = fmaf(__uint_as_float(q.x & 0xFFFF0000u), x[1], s);
            s = fmaf(__uint_as_float(q.y << 16), x[2], s); s = fmaf(__uint_as_float(q.y & 0xFFFF0000u), x[3], s);
            s = fmaf(__uint_as_float(q.z << 16), x[4], s); s = fmaf(__uint_as_float(q.z & 0xFFFF0000u), x[5], s);
            s = fmaf(__uint_as_float(q.w << 16), x[6], s); s = fmaf(__uint_as_float(q.w & 0xFFFF0000u), x[7], s);
        }
        acc[r] = wsum(s);
    }
    // 4 floats per workgroup feed the next launch (rows 0..3 of the workgroup)
    if (lane == 0) out[blockIdx.x * 4 + w] = acc[0] + acc[1] + acc[2] + acc[3] + acc[4] + acc[5];
    stamp_end(i, t0);
}

int main(int argc, char **argv) {
    // --quiet: no per-call trace; --no-attr: no hipFuncSetAttribute (64 KB of
    // dynamic LDS is within the default limit); --relaxed: capture in relaxed
    // mode instead of global
    // (under rocprofv3 --kernel-trace this tool faults in the 4th variant of a
    // run, whatever it is -- not the kernarg size: profiles/r06i_mb_launch_fault.txt;
    // profile at most three variants per run with --only)
    // --reps N: timed replays per variant (default 20); --only a,b: just these
    // variants (fewer dispatch records under the profiler)
    // --kernarg-sweep: only the x4k body through by-value structs of 128..1024 B
    // (ascending), each in graphs of --nodes N (default NL) launches -- under
    // rocprofv3 the first size that faults names the boundary (round 6, VERDICT
    // r05 #7)
    // --keep-graphs: keep every variant's graph (exec) alive until exit instead
    // of destroying it after the variant; --desc: the kernarg sweep largest first
    bool no_attr = false, relaxed = false, kb_sweep = false, keep = false, desc = false;
    int reps_arg = 20, nodes = NL;
    const char *only = nullptr;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--quiet")) g_trace = 0;
        if (!strcmp(argv[i], "--no-attr")) no_attr = true;
        if (!strcmp(argv[i], "--relaxed")) relaxed = true;
        if (!strcmp(argv[i], "--reps") && i + 1 < argc) reps_arg = atoi(argv[++i]);
        if (!strcmp(argv[i], "--only") && i + 1 < argc) only = argv[++i];
        if (!strcmp(argv[i], "--kernarg-sweep")) kb_sweep = true;
        if (!strcmp(argv[i], "--keep-graphs")) keep = true;
        if (!strcmp(argv[i], "--desc")) desc = true;
        if (!strcmp(argv[i], "--nodes") && i + 1 < argc) nodes = std::max(2, std::min(NL, atoi(argv[++i])));
    }
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float *va, *vb;
    CK(hipMalloc(&va, 8 * 16384 * 4));
    CK(hipMalloc(&vb, 8 * 16384 * 4));
    CK(hipMemset(va, 0, 8 * 16384 * 4));
    CK(hipMemset(vb, 0, 8 * 16384 * 4));
    uint16_t *W;
    const size_t wn = (size_t)6144 * 1024;
    CK(hipMalloc(&W, wn * 2));
    CK(hipMemset(W, 0x3c, wn * 2));
    if (!no_attr) CK(hipFuncSetAttribute((const void *)k_x4k_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
    static unsigned long long hs[NL][MAXG][2];

    std::vector<std::pair<hipGraph_t, hipGraphExec_t>> kept;
    auto run = [&](const char *name, int grid, auto launch) {
        if (only) {   // comma-separated exact names
            bool hit = false;
            const size_t n = strlen(name);
            for (const char *p = only; *p;) {
                const char *q = strchr(p, ',');
                const size_t m = q ? (size_t)(q - p) : strlen(p);
                if (m == n && !strncmp(p, name, n)) hit = true;
                if (!q) break;
                p = q + 1;
            }
            if (!hit) return;
        }
        hipGraph_t g;
        hipGraphExec_t ge;
        if (g_trace) fprintf(stderr, "[mb_launch] variant %s grid %d nodes %d\n", name, grid, nodes);
        CK(hipStreamBeginCapture(st, relaxed ? hipStreamCaptureModeRelaxed : hipStreamCaptureModeGlobal));
        for (int i = 0; i < nodes; ++i) launch(i);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int r = 0; r < 3; ++r) CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        const int reps = reps_arg;
        CK(hipEventRecord(e0, st));
        for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        // one more replay for the stamps
        CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        CK(hipMemcpyFromSymbol(hs, HIP_SYMBOL(g_st), sizeof(hs)));
        std::vector<double> span, gap, ramp;
        for (int i = 0; i < nodes; ++i) {
            unsigned long long s0 = ~0ull, s1 = 0, e1v = 0;
            for (int b = 0; b < grid; ++b) {
                s0 = std::min(s0, hs[i][b][0]);
                s1 = std::max(s1, hs[i][b][0]);
                e1v = std::max(e1v, hs[i][b][1]);
            }
            span.push_back((e1v - s0) * 0.01);
            ramp.push_back((s1 - s0) * 0.01);
            if (i + 1 < nodes) {
                unsigned long long n0 = ~0ull;
                for (int b = 0; b < grid; ++b) n0 = std::min(n0, hs[i + 1][b][0]);
                gap.push_back(((double)n0 - (double)e1v) * 0.01);
            }
        }
        auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v.empty() ? 0.0 : v[v.size() / 2]; };
        const bool stamped = hs[nodes / 2][0][1] != 0;
        printf("%-12s grid %3d: %6.2f us/kernel", name, grid, ms * 1e3 / (reps * nodes));
        fflush(stdout);
        if (stamped) printf("   span %5.2f  ramp %5.2f  gap %5.2f  (span+gap %5.2f)", med(span), med(ramp), med(gap),
                            med(span) + med(gap));
        printf("\n");
        memset(hs, 0, sizeof(hs));
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_st), hs, sizeof(hs)));
        if (keep) {
            kept.push_back({g, ge});
        } else {
            CK(hipGraphExecDestroy(ge));
            CK(hipGraphDestroy(g));
        }
    };
    auto pp = [&](int i, const float *&in, float *&out) { in = (i & 1) ? vb : va; out = (i & 1) ? va : vb; };
    if (kb_sweep) {
        auto kb = [&](auto bc) {
            constexpr int B = decltype(bc)::value;
            char nm[32];
            snprintf(nm, sizeof nm, "kb%d", B);
            run(nm, 256, [&](int i) { KB<B> a{}; a.i = i; pp(i, a.in, a.out);
                hipLaunchKernelGGL(k_x4k_kb<B>, dim3(256), dim3(256), 0, st, a); });
        };
        if (!desc) {
            kb(std::integral_constant<int, 128>{}); kb(std::integral_constant<int, 192>{});
            kb(std::integral_constant<int, 224>{}); kb(std::integral_constant<int, 232>{});
            kb(std::integral_constant<int, 240>{}); kb(std::integral_constant<int, 248>{});
            kb(std::integral_constant<int, 256>{}); kb(std::integral_constant<int, 264>{});
            kb(std::integral_constant<int, 288>{}); kb(std::integral_constant<int, 384>{});
            kb(std::integral_constant<int, 512>{}); kb(std::integral_constant<int, 1024>{});
        } else {
            kb(std::integral_constant<int, 1024>{}); kb(std::integral_constant<int, 512>{});
            kb(std::integral_constant<int, 384>{}); kb(std::integral_constant<int, 288>{});
            kb(std::integral_constant<int, 264>{}); kb(std::integral_constant<int, 256>{});
            kb(std::integral_constant<int, 128>{});
        }
        for (auto &k : kept) { CK(hipGraphExecDestroy(k.second)); CK(hipGraphDestroy(k.first)); }
        return 0;
    }
    for (int grid : {256, 512}) {
        run("empty", grid, [&](int) { hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, st); });
        run("stamp", grid, [&](int i) { hipLaunchKernelGGL(k_stamp, dim3(grid), dim3(256), 0, st, i); });
        run("x4k", grid, [&](int i) { const float *in; float *out; pp(i, in, out);
            hipLaunchKernelGGL(k_x4k, dim3(grid), dim3(256), 0, st, i, in, out); });
        run("x4k_big", grid, [&](int i) { Big b{}; b.i = i; pp(i, b.in, b.out);
                hipLaunchKernelGGL(k_x4k_big, dim3(grid), dim3(256), 0, st, b); });
        run("x4k_vgpr", grid, [&](int i) { const float *in; float *out; pp(i, in, out);
            hipLaunchKernelGGL(k_x4k_vgpr, dim3(grid), dim3(256), 0, st, i, in, out); });
        run("x4k_lds", grid, [&](int i) { const float *in; float *out; pp(i, in, out);
            hipLaunchKernelGGL(k_x4k_lds, dim3(grid), dim3(256), 65536, st, i, in, out); });
        run("x4k_code", grid, [&](int i) { const float *in; float *out; pp(i, in, out);
            hipLaunchKernelGGL(k_x4k_code<0>, dim3(grid), dim3(256), 0, st, i, in, out); });
        run("x4k_code4", grid, [&](int i) { const float *in; float *out; pp(i, in, out);   // 4 kernels rotating: 96 KB
            switch (i & 3) {
                case 0: hipLaunchKernelGGL(k_x4k_code<0>, dim3(grid), dim3(256), 0, st, i, in, out); break;
                case 1: hipLaunchKernelGGL(k_x4k_code<1>, dim3(grid), dim3(256), 0, st, i, in, out); break;
                case 2: hipLaunchKernelGGL(k_x4k_code<2>, dim3(grid), dim3(256), 0, st, i, in, out); break;
                default: hipLaunchKernelGGL(k_x4k_code<3>, dim3(grid), dim3(256), 0, st, i, in, out); break;
            } });
        run("x4k_loop", grid, [&](int i) { const float *in; float *out; pp(i, in, out);
            hipLaunchKernelGGL(k_x4k_loop, dim3(grid), dim3(256), 0, st, i, in, out); });
        run("x4k_resid", grid, [&](int i) { const float *in; float *out; pp(i, in, out);
            hipLaunchKernelGGL(k_x4k_resid, dim3(grid), dim3(256), 0, st, i, in, out); });
        if (grid == 256) {
            run("x32k", grid, [&](int i) { const float *in; float *out; pp(i, in, out);
                hipLaunchKernelGGL((k_xbig<32, 0>), dim3(grid), dim3(256), 0, st, i, in, out); });
            run("x32k_rep8", grid, [&](int i) { const float *in; float *out; pp(i, in, out);
                hipLaunchKernelGGL((k_xbig<32, 1>), dim3(grid), dim3(256), 0, st, i, in, out); });
            run("x64k", grid, [&](int i) { const float *in; float *out; pp(i, in, out);
                hipLaunchKernelGGL((k_xbig<64, 0>), dim3(grid), dim3(256), 0, st, i, in, out); });
            run("x64k_rep8", grid, [&](int i) { const float *in; float *out; pp(i, in, out);
                hipLaunchKernelGGL((k_xbig<64, 1>), dim3(grid), dim3(256), 0, st, i, in, out); });
        }
        if (grid == 256)
            run("gemv_gu", grid, [&](int i) { const float *in; float *out; pp(i, in, out);
                hipLaunchKernelGGL(k_gemv_gu, dim3(grid), dim3(256), 0, st, i, W, in, out); });
    }
    return 0;
}
