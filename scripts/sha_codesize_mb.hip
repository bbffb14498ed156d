// sha_codesize_mb.hip — is the SHA-256 compression bound by its code size?  Register-resident
// data, 4 waves per SIMD, every CU; the production compression (64 rounds unrolled: ~11.5 KB of
// code per block) against the same rounds rolled into a loop of R-round bodies (R = 16 / 32),
// with the round constants read per iteration by scalar loads.  Same digests (checked).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/sha_codesize_mb.hip -o build/sha_cs
#include "../sdfs_amd/csrc/cdc_kernels.hip"

#include <cstdio>

using namespace sdfs;

__constant__ uint32_t cK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

// Rounds 16*it .. 16*it+15 of the 64 (R = 16) with the schedule of rounds 16..63 computed at the
// head of iterations 1..3, as sha256_compress does per 16 rounds.
template <int R>
__device__ __forceinline__ void sha256_compress_rolled(uint32_t (&s)[8], uint32_t (&w)[16]) {
    uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll 1
    for (int it = 0; it < 64 / R; it++) {
        const uint32_t* K = cK + R * it;
#pragma unroll
        for (int i = 0; i < R; i++) {
            if ((i & 15) == 0 && (it > 0 || i > 0)) {
#pragma unroll
                for (int j = 0; j < 16; j++) {
                    const uint32_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
                    const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
                    const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
                    w[j] = w[j] + s0 + w[(j + 9) & 15] + s1;
                }
            }
            const uint32_t wi = w[i & 15];
            const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
            const uint32_t ch = (e & f) | (~e & g);
            const uint32_t t1 = h + S1 + ch + K[i] + wi;
            const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
            const uint32_t mj = maj3(a, b, c);
            h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
        }
    }
    s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
}


// Two independent compressions per lane, their rounds interleaved (ILP 2 per lane).
__device__ __forceinline__ void sha256_compress2(uint32_t (&s)[8], uint32_t (&w)[16], uint32_t (&s2)[8],
                                                 uint32_t (&w2)[16]) {
    uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
    uint32_t A = s2[0], B = s2[1], C = s2[2], D = s2[3], E = s2[4], F = s2[5], G = s2[6], H = s2[7];
#pragma unroll 1
    for (int it = 0; it < 4; it++) {
        const uint32_t* K = cK + 16 * it;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            if (i == 0 && it > 0) {
#pragma unroll
                for (int j = 0; j < 16; j++) {
                    uint32_t w15 = w[(j + 1) & 15], w2_ = w[(j + 14) & 15];
                    w[j] = w[j] + xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3) + w[(j + 9) & 15] +
                           xor3(rotr(w2_, 17), rotr(w2_, 19), w2_ >> 10);
                    w15 = w2[(j + 1) & 15]; w2_ = w2[(j + 14) & 15];
                    w2[j] = w2[j] + xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3) + w2[(j + 9) & 15] +
                            xor3(rotr(w2_, 17), rotr(w2_, 19), w2_ >> 10);
                }
            }
            {
                const uint32_t t1 = h + xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)) + ((e & f) | (~e & g)) + K[i] + w[i];
                const uint32_t t2 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)) + maj3(a, b, c);
                h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
            }
            {
                const uint32_t t1 = H + xor3(rotr(E, 6), rotr(E, 11), rotr(E, 25)) + ((E & F) | (~E & G)) + K[i] + w2[i];
                const uint32_t t2 = xor3(rotr(A, 2), rotr(A, 13), rotr(A, 22)) + maj3(A, B, C);
                H = G; G = F; F = E; E = D + t1; D = C; C = B; B = A; A = t1 + t2;
            }
        }
    }
    s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
    s2[0] += A; s2[1] += B; s2[2] += C; s2[3] += D; s2[4] += E; s2[5] += F; s2[6] += G; s2[7] += H;
}

__global__ __launch_bounds__(256) void ksha2(uint32_t* out, int blocks_per_lane) {
    extern __shared__ uint32_t pad[];
    uint32_t s[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint32_t s2[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint32_t seed = blockIdx.x * 256 + threadIdx.x;
    for (int b = 0; b < blocks_per_lane; b += 2) {
        uint32_t w[16], w2[16];
#pragma unroll
        for (int j = 0; j < 16; j++) { w[j] = s[j & 7] + seed + j; w2[j] = s2[j & 7] + seed + 3 * j; }
        sha256_compress2(s, w, s2, w2);
    }
    if (threadIdx.x == 1023) pad[0] = s[0];
    out[blockIdx.x * 256 + threadIdx.x] = s[0] ^ s[1] ^ s[2] ^ s[3] ^ s[4] ^ s[5] ^ s[6] ^ s[7] ^ s2[0];
}

static double run2(uint32_t* out, int cus, int wps, int bpl, int reps) {
    const size_t lds = (160 * 1024) / wps - 1024;
    const int blocks = cus * wps * 4;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(ksha2, dim3(blocks), dim3(256), lds, 0, out, bpl);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(ksha2, dim3(blocks), dim3(256), lds, 0, out, bpl);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    return (double)blocks * 256 * bpl * 64 * reps / ms / 1e6;
}

template <int FORM>
__global__ __launch_bounds__(256) void ksha(uint32_t* out, int blocks_per_lane) {
    extern __shared__ uint32_t pad[];
    uint32_t s[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint32_t seed = blockIdx.x * 256 + threadIdx.x;
    for (int b = 0; b < blocks_per_lane; b++) {
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; j++) w[j] = s[j & 7] + seed + j;
        if constexpr (FORM == 0)
            sha256_compress(s, w);
        else
            sha256_compress_rolled<FORM>(s, w);
    }
    if (threadIdx.x == 1023) pad[0] = s[0];
    out[blockIdx.x * 256 + threadIdx.x] = s[0] ^ s[1] ^ s[2] ^ s[3] ^ s[4] ^ s[5] ^ s[6] ^ s[7];
}

template <int FORM>
static double run(uint32_t* out, int cus, int wps, int bpl, int reps) {
    const size_t lds = (160 * 1024) / wps - 1024;
    const int blocks = cus * wps * 4;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(ksha<FORM>, dim3(blocks), dim3(256), lds, 0, out, bpl);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(ksha<FORM>, dim3(blocks), dim3(256), lds, 0, out, bpl);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    return (double)blocks * 256 * bpl * 64 * reps / ms / 1e6;  // GB/s
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    uint32_t *out, *ref;
    (void)hipMalloc(&out, 64 << 20);
    (void)hipMalloc(&ref, 64 << 20);
    const int bpl = 100, wps = 4, n = cus * wps * 4 * 256;
    // correctness: the rolled forms give the production digests
    hipLaunchKernelGGL(ksha<0>, dim3(cus * wps * 4), dim3(256), (160 * 1024) / wps - 1024, 0, ref, 3);
    for (int f : {16, 32}) {
        if (f == 16) hipLaunchKernelGGL(ksha<16>, dim3(cus * wps * 4), dim3(256), (160 * 1024) / wps - 1024, 0, out, 3);
        else hipLaunchKernelGGL(ksha<32>, dim3(cus * wps * 4), dim3(256), (160 * 1024) / wps - 1024, 0, out, 3);
        (void)hipDeviceSynchronize();
        std::vector<uint32_t> x(n), y(n);
        (void)hipMemcpy(x.data(), ref, 4ull * n, hipMemcpyDeviceToHost);
        (void)hipMemcpy(y.data(), out, 4ull * n, hipMemcpyDeviceToHost);
        printf("rolled %d: %s\n", f, x == y ? "same digests" : "DIFFERENT");
    }
    for (int rep = 0; rep < 3; rep++)
        printf("unrolled %.1f GB/s | rolled16 %.1f | rolled32 %.1f\n", run<0>(out, cus, wps, bpl, 5),
               run<16>(out, cus, wps, bpl, 5), run<32>(out, cus, wps, bpl, 5));
    for (int w2 : {1, 2, 3, 4})
        printf("two chains per lane, %d waves/SIMD: %.1f GB/s\n", w2, run2(out, cus, w2, bpl, 5));
    for (int w1 : {1, 2, 3, 4, 6, 8})
        printf("one chain per lane, %d waves/SIMD: %.1f GB/s\n", w1, run<16>(out, cus, w1, bpl, 5));
    return 0;
}
