// Probe of gfx950 LDS-DMA (buffer_load_dwordx4 ... lds) semantics the halo conv's weight loader relies on:
//   1. destination = M0 + instruction offset + 16 * lane (one wave-instruction writes 1 KiB contiguously);
//   2. M0 bases above 64 KiB reach the upper LDS (160 KiB per CU on MI355X);
//   3. an out-of-range buffer offset writes zeros into the lane's 16 B (and moves no data).
// Build: hipcc --offload-arch=gfx950 -O3 -o build_ab/lds_dma_probe tools/lds_dma_probe.hip
// Run on the GPU box; prints one line per probed base and PASS / FAIL.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int LDS_BYTES = 152 * 1024;

__global__ __launch_bounds__(64) void k_probe(const unsigned* __restrict__ src, unsigned* __restrict__ out, int base,
                                              int nsrc_bytes) {
    __shared__ __attribute__((aligned(16))) unsigned lds[LDS_BYTES / 4];
    const int lane = threadIdx.x;
    // poison the region so a dropped write is visible
    for (int i = lane; i < LDS_BYTES / 4; i += 64) lds[i] = 0xdeadbeefu;
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, nsrc_bytes, 0x00020000);
    // lane l reads source 16-B piece (63 - l): a reversed gather; lane 5 is out of range
    const unsigned voff = lane == 5 ? 0x80000000u : (unsigned)(63 - lane) * 16u;
    const unsigned m0v = (unsigned)(uintptr_t)lds + (unsigned)base;
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %1, %3, 0 offen offset:16 lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(m0v), "s"(rs)
        : "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // copy back 1 KiB + 64 B around the destination (base - 16 .. base + 1024 + 48)
    for (int i = lane; i < (1024 + 64) / 4; i += 64) out[i] = lds[(base - 16) / 4 + i];
}

int main() {
    std::vector<unsigned> h(64 * 4 + 16);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0x1000u + (unsigned)i;
    unsigned *d_src, *d_out;
    hipMalloc(&d_src, h.size() * 4);
    hipMalloc(&d_out, 1088);
    hipMemcpy(d_src, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    const int bases[] = {16, 1024, 32768, 65536 - 512, 65536, 98304, 131072, LDS_BYTES - 1024 - 64};
    bool all = true;
    for (int base : bases) {
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, d_src, d_out, base, (int)(h.size() * 4));
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("base %d: launch failed\n", base);
            return 2;
        }
        std::vector<unsigned> o(1088 / 4);
        hipMemcpy(o.data(), d_out, 1088, hipMemcpyDeviceToHost);
        // expected: 16 B poison, then (with instruction offset 16) piece 0 at +16: the 16 B at base + 16 + 16*l
        // hold source piece (63 - l) shifted by the offset: src byte (63 - l)*16 + 16
        int bad = 0, zero_ok = 1, shift = -1;
        // find where lane 0's data landed: search for src word index (63*4 + 4)
        for (int i = 0; i < 1088 / 4; ++i)
            if (o[i] == 0x1000u + 63 * 4 + 4) {
                shift = i * 4 - 16;  // bytes from base
                break;
            }
        if (shift < 0) {
            printf("base %d: lane 0 data not found\n", base);
            all = false;
            continue;
        }
        for (int l = 0; l < 64; ++l)
            for (int j = 0; j < 4; ++j) {
                const int idx = (16 + shift + 16 * l) / 4 + j;
                if (idx >= 1088 / 4) { bad++; continue; }
                const unsigned want = l == 5 ? 0u : 0x1000u + (unsigned)((63 - l) * 4 + 4 + j);
                if (o[idx] != want) {
                    if (l == 5) zero_ok = 0;
                    bad++;
                }
            }
        const bool poison_before = o[(16 + shift) / 4 - 1] == 0xdeadbeefu;
        printf("base %6d: dest offset from M0 = %d B, mismatches %d, OOB lane zeros %s, word before intact %s\n", base,
               shift, bad, zero_ok ? "yes" : "no", poison_before ? "yes" : "no");
        if (bad || shift != 16) all = false;
    }
    printf("%s\n", all ? "PASS" : "FAIL");
    return all ? 0 : 1;
}
