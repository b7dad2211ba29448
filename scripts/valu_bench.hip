// valu_bench.hip -- issue cost of the vector instructions the Rice kernel's
// phase 1 and packer are made of, on this box: each kernel runs 8 independent
// chains of one instruction, 64 deep, in inline asm, and reports shader-clock
// cycles (s_memtime) per wave-instruction at 1 and at 4 waves per SIMD.
// Not part of the product (scripts/).
//   hipcc --offload-arch=gfx950 -O3 -o exp/bin/valu_bench scripts/valu_bench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define R8(x) x x x x x x x x
// each wave runs its 512-instruction body NREP times, so that the waves of a
// launch overlap for most of their lives (all are resident from the start)
#define NREP 32
#define BODY(ins) R8(R8(ins))

#define KERN(name, ins, cons)                                                                      \
	__global__ __launch_bounds__(256) void name(uint64_t *out, uint32_t seed)                  \
	{                                                                                          \
		uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u;          \
		uint32_t b0 = a0 ^ 9u, b1 = a1 ^ 9u, b2 = a2 ^ 9u, b3 = a3 ^ 9u;                     \
		uint32_t c0 = 3u, c1 = 5u, c2 = 7u, c3 = 11u;                                          \
		__syncthreads();                                                                   \
		const uint64_t t0 = __builtin_amdgcn_s_memtime();                                  \
		for (int rep = 0; rep < NREP; rep++)                                               \
			asm volatile(BODY(ins) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(b0), "+v"(b1), \
				     "+v"(b2), "+v"(b3)                                                    \
				     : cons(c0), cons(c1), cons(c2), cons(c3));                            \
		const uint64_t t1 = __builtin_amdgcn_s_memtime();                                  \
		if ((threadIdx.x & 63u) == 0u)                                                     \
			out[blockIdx.x * 4u + threadIdx.x / 64u] = t1 - t0;                        \
		if (a0 + a1 + a2 + a3 + b0 + b1 + b2 + b3 == 0x12345u)                             \
			out[0] = 1;                                                                \
	}

#define V "v"
// 8 instructions per line, one per chain (operands %0..%7 are the chains,
// %8..%11 constant inputs)
KERN(k_add, "v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %9\n v_add_u32 %2, %2, %10\n v_add_u32 %3, %3, %11\n"
	    "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %9\n v_add_u32 %6, %6, %10\n v_add_u32 %7, %7, %11\n", V)
// the same VOP2 add with a 32-bit literal (an 8-byte encoding) and as VOP3 (_e64, 8 bytes)
KERN(k_add_lit, "v_add_u32 %0, 0x12345, %0\n v_add_u32 %1, 0x12345, %1\n v_add_u32 %2, 0x12345, %2\n v_add_u32 %3, 0x12345, %3\n"
		"v_add_u32 %4, 0x12345, %4\n v_add_u32 %5, 0x12345, %5\n v_add_u32 %6, 0x12345, %6\n v_add_u32 %7, 0x12345, %7\n", V)
KERN(k_add_e64, "v_add_u32_e64 %0, %0, %8\n v_add_u32_e64 %1, %1, %9\n v_add_u32_e64 %2, %2, %10\n v_add_u32_e64 %3, %3, %11\n"
		"v_add_u32_e64 %4, %4, %8\n v_add_u32_e64 %5, %5, %9\n v_add_u32_e64 %6, %6, %10\n v_add_u32_e64 %7, %7, %11\n", V)
// alternating 4-byte and 8-byte instructions
KERN(k_mix, "v_add_u32 %0, %0, %8\n v_lshl_or_b32 %1, %1, %9, %10\n v_add_u32 %2, %2, %10\n v_lshl_or_b32 %3, %3, %11, %8\n"
	    "v_add_u32 %4, %4, %8\n v_lshl_or_b32 %5, %5, %9, %10\n v_add_u32 %6, %6, %10\n v_lshl_or_b32 %7, %7, %11, %8\n", V)
KERN(k_lshl_or, "v_lshl_or_b32 %0, %0, %8, %9\n v_lshl_or_b32 %1, %1, %9, %10\n v_lshl_or_b32 %2, %2, %10, %11\n"
		"v_lshl_or_b32 %3, %3, %11, %8\n v_lshl_or_b32 %4, %4, %8, %9\n v_lshl_or_b32 %5, %5, %9, %10\n"
		"v_lshl_or_b32 %6, %6, %10, %11\n v_lshl_or_b32 %7, %7, %11, %8\n", V)
KERN(k_alignbit, "v_alignbit_b32 %0, %0, %4, %8\n v_alignbit_b32 %1, %1, %5, %9\n v_alignbit_b32 %2, %2, %6, %10\n"
		 "v_alignbit_b32 %3, %3, %7, %11\n v_alignbit_b32 %4, %4, %0, %8\n v_alignbit_b32 %5, %5, %1, %9\n"
		 "v_alignbit_b32 %6, %6, %2, %10\n v_alignbit_b32 %7, %7, %3, %11\n", V)
// 64-bit operations: four 64-bit chains
#define KERN64(name, ins)                                                                          \
	__global__ __launch_bounds__(256) void name(uint64_t *out, uint32_t seed)                  \
	{                                                                                          \
		uint64_t a0 = seed + threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u;          \
		uint32_t c0 = 3u, c1 = 5u;                                                         \
		__syncthreads();                                                                   \
		const uint64_t t0 = __builtin_amdgcn_s_memtime();                                  \
		for (int rep = 0; rep < NREP; rep++)                                               \
			asm volatile(BODY(ins) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(c0), "v"(c1)); \
		const uint64_t t1 = __builtin_amdgcn_s_memtime();                                  \
		if ((threadIdx.x & 63u) == 0u)                                                     \
			out[blockIdx.x * 4u + threadIdx.x / 64u] = t1 - t0;                        \
		if (a0 + a1 + a2 + a3 == 0x12345u)                                                 \
			out[0] = 1;                                                                \
	}
KERN64(k_lshl64, "v_lshlrev_b64 %0, %4, %0\n v_lshlrev_b64 %1, %5, %1\n v_lshlrev_b64 %2, %4, %2\n"
		 "v_lshlrev_b64 %3, %5, %3\n v_lshlrev_b64 %0, %5, %0\n v_lshlrev_b64 %1, %4, %1\n"
		 "v_lshlrev_b64 %2, %5, %2\n v_lshlrev_b64 %3, %4, %3\n")
KERN64(k_lshladd64, "v_lshl_add_u64 %0, %0, 1, %1\n v_lshl_add_u64 %1, %1, 1, %2\n v_lshl_add_u64 %2, %2, 1, %3\n"
		    "v_lshl_add_u64 %3, %3, 1, %0\n v_lshl_add_u64 %0, %0, 1, %1\n v_lshl_add_u64 %1, %1, 1, %2\n"
		    "v_lshl_add_u64 %2, %2, 1, %3\n v_lshl_add_u64 %3, %3, 1, %0\n")
KERN(k_bfe, "v_bfe_u32 %0, %0, 8, 8\n v_bfe_u32 %1, %1, 8, 8\n v_bfe_u32 %2, %2, 8, 8\n v_bfe_u32 %3, %3, 8, 8\n"
	    "v_bfe_u32 %4, %4, 8, 8\n v_bfe_u32 %5, %5, 8, 8\n v_bfe_u32 %6, %6, 8, 8\n v_bfe_u32 %7, %7, 8, 8\n", V)
KERN(k_pkadd, "v_pk_add_u16 %0, %0, %8\n v_pk_add_u16 %1, %1, %9\n v_pk_add_u16 %2, %2, %10\n v_pk_add_u16 %3, %3, %11\n"
	      "v_pk_add_u16 %4, %4, %8\n v_pk_add_u16 %5, %5, %9\n v_pk_add_u16 %6, %6, %10\n v_pk_add_u16 %7, %7, %11\n", V)
KERN(k_sdwa, "v_lshlrev_b32_sdwa %0, %8, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"
	     "v_lshlrev_b32_sdwa %1, %9, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"
	     "v_lshlrev_b32_sdwa %2, %10, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"
	     "v_lshlrev_b32_sdwa %3, %11, %3 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"
	     "v_lshlrev_b32_sdwa %4, %8, %4 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"
	     "v_lshlrev_b32_sdwa %5, %9, %5 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"
	     "v_lshlrev_b32_sdwa %6, %10, %6 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n"
	     "v_lshlrev_b32_sdwa %7, %11, %7 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n", V)
KERN(k_sad, "v_sad_u8 %0, %0, 0, %8\n v_sad_u8 %1, %1, 0, %9\n v_sad_u8 %2, %2, 0, %10\n v_sad_u8 %3, %3, 0, %11\n"
	    "v_sad_u8 %4, %4, 0, %8\n v_sad_u8 %5, %5, 0, %9\n v_sad_u8 %6, %6, 0, %10\n v_sad_u8 %7, %7, 0, %11\n", V)
KERN(k_cvt, "v_cvt_f32_u32 %0, %0\n v_cvt_f32_u32 %1, %1\n v_cvt_f32_u32 %2, %2\n v_cvt_f32_u32 %3, %3\n"
	    "v_cvt_f32_u32 %4, %4\n v_cvt_f32_u32 %5, %5\n v_cvt_f32_u32 %6, %6\n v_cvt_f32_u32 %7, %7\n", V)
// LDS: ds_or_b32 to lane-private words (no return), 8 per line
__global__ __launch_bounds__(256) void k_dsor(uint64_t *out, uint32_t seed)
{
	__shared__ uint32_t L[256 * 9];
	for (uint32_t i = threadIdx.x; i < 256 * 9; i += 256)
		L[i] = 0;
	__syncthreads();
	uint32_t ad = (uint32_t)(uintptr_t)&L[threadIdx.x * 9u], v = seed + threadIdx.x;
	const uint64_t t0 = __builtin_amdgcn_s_memtime();
	for (int rep = 0; rep < NREP; rep++)
	asm volatile(BODY("ds_or_b32 %0, %1\n ds_or_b32 %0, %1 offset:4\n ds_or_b32 %0, %1 offset:8\n"
			  "ds_or_b32 %0, %1 offset:12\n ds_or_b32 %0, %1 offset:16\n ds_or_b32 %0, %1 offset:20\n"
			  "ds_or_b32 %0, %1 offset:24\n ds_or_b32 %0, %1 offset:28\n") "s_waitcnt lgkmcnt(0)\n"
		     :
		     : "v"(ad), "v"(v)
		     : "memory");
	const uint64_t t1 = __builtin_amdgcn_s_memtime();
	if ((threadIdx.x & 63u) == 0u)
		out[blockIdx.x * 4u + threadIdx.x / 64u] = t1 - t0;
}

typedef void (*kfn)(uint64_t *, uint32_t);

int main()
{
	uint64_t *d;
	const int maxb = 256 * 8;  // (up to 6 waves per SIMD)
	hipMalloc(&d, maxb * 4 * 8);
	struct K {
		const char *name;
		kfn f;
	} ks[] = {{"v_add_u32", k_add}, {"v_add_u32 literal", k_add_lit}, {"v_add_u32_e64", k_add_e64}, {"add / lshl_or mix", k_mix},          {"v_lshl_or_b32", k_lshl_or}, {"v_alignbit_b32", k_alignbit},
		  {"v_lshlrev_b64", k_lshl64},   {"v_bfe_u32", k_bfe},         {"v_pk_add_u16", k_pkadd},
		  {"v_lshlrev_sdwa", k_sdwa},    {"v_sad_u8", k_sad},          {"v_cvt_f32_u32", k_cvt},
		  {"v_lshl_add_u64", k_lshladd64}, {"ds_or_b32", k_dsor}};
	uint64_t h[maxb * 4];
	for (auto &k : ks) {
		for (int wps : {1, 2, 4, 6}) {
			// 256-thread blocks = one wave per SIMD each; wps blocks per CU
			const int nb = 256 * wps;
			for (int rep = 0; rep < 3; rep++) {
				hipLaunchKernelGGL(k.f, dim3(nb), dim3(256), 0, 0, d, 1u + rep);
				hipDeviceSynchronize();
			}
			hipMemcpy(h, d, nb * 4 * 8, hipMemcpyDeviceToHost);
			double s = 0;
			for (int i = 0; i < nb * 4; i++)
				s += (double)h[i];
			printf("%-16s waves/SIMD %d: %6.2f cycles per wave-instruction\n", k.name, wps, s / (nb * 4) / (512.0 * NREP));
		}
	}
	return 0;
}
