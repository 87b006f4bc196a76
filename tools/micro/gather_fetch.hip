// FETCH_SIZE calibration for the rollout kernel's access pattern: 2-byte loads scattered over a
// 512^3 field of 16-bit d^2 (256 MiB, cfg4's field).  Every kernel below touches a KNOWN set of
// 128-B lines (or 64-B / 32-B pieces of them) exactly once per launch, so rocprofv3's FETCH_SIZE
// per dispatch divided by the count of lines touched gives the bytes the counter tallies per
// line for this pattern -- the correction factor the rollout's traffic figures need
// (MI355X_MICROARCH.md:298 calibrates x2 for 16-B-per-lane streaming reads only).
//
// Kernels (launch order = the order of the lines of known.json):
//   k_stream16      16 B per lane, coalesced, over the whole field: the guide's calibration
//   k_line1         one 2-B load per 128-B line, the lines a bijective scatter of the field
//   k_line4         four 2-B loads per line by four neighbouring lanes (the rollout's lanes of
//                   one sphere at neighbouring waypoints often share a line)
//   k_half1         one 2-B load per 64-B half-line, every half of the touched lines (two
//                   requests per line, far apart in time)
//   k_sector1       one 2-B load per 32-B sector, every sector of the touched lines
// Each kernel runs twice: after an eviction pass (a 1 GiB streaming read: the field is not in
// the 256-MiB Infinity Cache, "cold") and right after the cold run ("warm": the touched lines
// are on-die).  Nothing is stored except on an impossible sum, so WRITE_SIZE stays ~0.
//
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/micro/gather_fetch tools/micro/gather_fetch.hip
// Run:   rocprofv3 --pmc FETCH_SIZE --output-format csv -d DIR -o p1 -- tools/micro/gather_fetch DIR/known.json
//        (tools/gpu.sh micro), then python3 tools/micro/gather_fetch.py DIR
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

constexpr size_t kFieldBytes = 512ull * 512 * 512 * 2;   // 256 MiB
constexpr uint32_t kLines = kFieldBytes / 128;           // 2^21
constexpr uint32_t kPerm = 0x9E3779B1u;                  // odd: g -> g * kPerm mod 2^k is a bijection

// line index of the g-th touched line: a bijective scatter of [0, nlines) over [0, kLines)
__device__ __forceinline__ uint32_t scatter(uint32_t g) { return (g * kPerm) & (kLines - 1); }

__global__ void k_stream16(const uint4* f, size_t n16, unsigned* out)
{
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = f[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u) out[0] = acc;
}

// one u16 per line: thread g reads lane-dependent word (g & 63) of line scatter(g)
__global__ void k_line1(const unsigned short* f, uint32_t nlines, unsigned* out)
{
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nlines) return;
    const unsigned v = f[(size_t)scatter(g) * 64 + (g & 63)];
    if (v == 0xfffeu) out[0] = v;
}

// four u16 of one line by four neighbouring lanes (words 0, 16, 32, 48 of the line)
__global__ void k_line4(const unsigned short* f, uint32_t nlines, unsigned* out)
{
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= 4 * nlines) return;
    const unsigned v = f[(size_t)scatter(g >> 2) * 64 + 16 * (g & 3)];
    if (v == 0xfffeu) out[0] = v;
}

// one u16 per 64-B half of each touched line: thread g < nlines reads half 0 of line scatter(g),
// thread nlines + g half 1 (the two requests of a line come from waves far apart)
__global__ void k_half1(const unsigned short* f, uint32_t nlines, unsigned* out)
{
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= 2 * nlines) return;
    const uint32_t h = g / nlines, l = g - h * nlines;
    const unsigned v = f[(size_t)scatter(l) * 64 + 32 * h + (l & 31)];
    if (v == 0xfffeu) out[0] = v;
}

// one u16 per 32-B sector of each touched line (four requests per line, far apart)
__global__ void k_sector1(const unsigned short* f, uint32_t nlines, unsigned* out)
{
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= 4 * nlines) return;
    const uint32_t s = g / nlines, l = g - s * nlines;
    const unsigned v = f[(size_t)scatter(l) * 64 + 16 * s + (l & 15)];
    if (v == 0xfffeu) out[0] = v;
}

// eviction pass: a 1 GiB streaming read (4x the Infinity Cache)
__global__ void k_evict(const uint4* f, size_t n16, unsigned* out)
{
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = f[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 0x9e3779b9u) out[1] = acc;
}

int main(int argc, char** argv)
{
    const char* known = argc > 1 ? argv[1] : "known.json";
    unsigned short* field;
    uint4* ev;
    unsigned* out;
    const size_t evb = 1ull << 30;
    CHECK(hipMalloc(&field, kFieldBytes));
    CHECK(hipMalloc(&ev, evb));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(field, 0x11, kFieldBytes));
    CHECK(hipMemset(ev, 0x22, evb));
    CHECK(hipMemset(out, 0, 64));
    const uint32_t nl = 1u << 20;   // lines touched by the gather kernels (half the field's lines)
    FILE* kf = fopen(known, "w");
    if (!kf) {
        perror(known);
        return 1;
    }
    fprintf(kf, "[\n");
    bool first = true;
    auto note = [&](const char* kernel, const char* temp, double lines, double requests, double bytes_loaded) {
        fprintf(kf, "%s {\"kernel\": \"%s\", \"cache\": \"%s\", \"lines\": %.0f, \"requests\": %.0f, \"bytes_loaded\": %.0f}",
                first ? "" : ",\n", kernel, temp, lines, requests, bytes_loaded);
        first = false;
    };
    auto evict = [&]() {
        hipLaunchKernelGGL(k_evict, dim3(4096), dim3(256), 0, 0, (const uint4*)ev, evb / 16, out);
        CHECK(hipGetLastError());
    };
    const int tb = 256;
    for (int rep = 0; rep < 2; ++rep) {   // rep 0 cold (after an eviction pass), rep 1 warm
        const char* temp = rep ? "warm" : "cold";
        if (!rep) evict();
        hipLaunchKernelGGL(k_stream16, dim3(4096), dim3(tb), 0, 0, (const uint4*)field, kFieldBytes / 16, out);
        note("k_stream16", temp, kLines, kLines, kFieldBytes);
    }
    struct G { const char* name; void (*fn)(const unsigned short*, uint32_t, unsigned*); uint32_t threads; double req_per_line; };
    const G gs[] = {{"k_line1", k_line1, nl, 1}, {"k_line4", k_line4, 4 * nl, 4}, {"k_half1", k_half1, 2 * nl, 2},
                    {"k_sector1", k_sector1, 4 * nl, 4}};
    for (const G& g : gs) {
        for (int rep = 0; rep < 2; ++rep) {
            const char* temp = rep ? "warm" : "cold";
            if (!rep) evict();
            hipLaunchKernelGGL(g.fn, dim3((g.threads + tb - 1) / tb), dim3(tb), 0, 0, (const unsigned short*)field, nl, out);
            CHECK(hipGetLastError());
            note(g.name, temp, nl, nl * g.req_per_line, 2.0 * nl * g.req_per_line);
        }
    }
    CHECK(hipDeviceSynchronize());
    fprintf(kf, "\n]\n");
    fclose(kf);
    unsigned h[2];
    CHECK(hipMemcpy(h, out, 8, hipMemcpyDeviceToHost));
    printf("gather_fetch done (%u %u), known counts in %s\n", h[0], h[1], known);
    CHECK(hipFree(field));
    CHECK(hipFree(ev));
    CHECK(hipFree(out));
    return 0;
}
