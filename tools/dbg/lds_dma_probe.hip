// Probe (diagnostic) of buffer_load_dword ... lds on gfx950:
//  (1) a lane whose offset is past the descriptor's byte range: does the DMA
//      write 0 into LDS or leave the word?
//  (2) the instruction offset: does it move the LDS address too, or only the
//      memory address?  (five loads, offsets 0..1024, M0 stepped by 256 as
//      k_synth's is[] prefetch does, then the same loads with M0 fixed)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ void k(const unsigned *src, unsigned *out, int mode) {
    __shared__ unsigned s[1600];
    const int lane = threadIdx.x;
    for (int i = lane; i < 1600; i += 64) s[i] = 0xAAAAAAAAu;
    __syncthreads();
    const unsigned long long a = (unsigned long long)src;
    u32x4 rs = {(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)a),
                (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(a >> 32)) & 0xFFFFu, 1100u, 0x00020000u};
    const unsigned lds0 = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned long long)(__attribute__((address_space(3))) unsigned *)s);
    unsigned keep;
    const int lo = lane * 4;
    if (mode == 0)
        __asm__ volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                         "buffer_load_dword %1, %3, 0 offen lds\n\ts_add_u32 m0, m0, 0x100\n\ts_nop 0\n\t"
                         "buffer_load_dword %1, %3, 0 offen offset:256 lds\n\ts_add_u32 m0, m0, 0x100\n\ts_nop 0\n\t"
                         "buffer_load_dword %1, %3, 0 offen offset:512 lds\n\ts_add_u32 m0, m0, 0x100\n\ts_nop 0\n\t"
                         "buffer_load_dword %1, %3, 0 offen offset:768 lds\n\ts_add_u32 m0, m0, 0x100\n\ts_nop 0\n\t"
                         "buffer_load_dword %1, %3, 0 offen offset:1024 lds\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(lo), "s"(lds0), "s"(rs) : "memory");
    else
        __asm__ volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                         "buffer_load_dword %1, %3, 0 offen offset:256 lds\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(lo), "s"(lds0), "s"(rs) : "memory");
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
    for (int i = lane; i < 1600; i += 64) out[i] = s[i];
}
int main() {
    static unsigned h[1600], o[1600];
    unsigned *d, *od;
    for (int i = 0; i < 1600; i++) h[i] = 1000 + i;
    if (hipMalloc(&d, sizeof h) || hipMalloc(&od, sizeof h)) return 2;
    (void)hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    for (int mode = 0; mode < 2; mode++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, od, mode);
        (void)hipMemcpy(o, od, sizeof o, hipMemcpyDeviceToHost);
        printf("mode %d:", mode);
        for (int w : {0, 1, 63, 64, 65, 128, 200, 256, 274, 275, 276, 300, 320}) printf(" s[%d]=%x", w, o[w]);
        printf("\n");
    }
    return 0;
}
