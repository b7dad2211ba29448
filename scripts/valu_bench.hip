// VALU issue-rate micro-benchmark for the integer ops the encoder uses.
// Each thread runs ITER iterations of 8 independent chains of one op; the
// grid puts WPS waves on every SIMD.  Reports cycles per wave-instruction per
// SIMD (clock from the device attribute).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define ITER 4096

#define CHAINS(OPSTR)                                                                                  \
	for (int i = 0; i < ITER; i++) {                                                               \
		asm volatile(OPSTR " %0, %0, %8\n\t" OPSTR " %1, %1, %8\n\t" OPSTR " %2, %2, %8\n\t" OPSTR \
			     " %3, %3, %8\n\t" OPSTR " %4, %4, %8\n\t" OPSTR " %5, %5, %8\n\t" OPSTR        \
			     " %6, %6, %8\n\t" OPSTR " %7, %7, %8"                                          \
			     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
			     : "v"(k));                                                                     \
	}

template <int OP>
__global__ void bench(uint32_t *out, uint32_t k)
{
	uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
		 a7 = a0 + 7;
	if (OP == 0) {
		CHAINS("v_add_u32")
	} else if (OP == 1) {
		CHAINS("v_xor_b32")
	} else if (OP == 2) {
		CHAINS("v_pk_add_u16")
	} else if (OP == 3) {
		CHAINS("v_bfm_b32")
	} else if (OP == 5) {
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_alignbit_b32 %0, %0, %1, %8\n\tv_alignbit_b32 %1, %1, %2, %8\n\t"
				     "v_alignbit_b32 %2, %2, %3, %8\n\tv_alignbit_b32 %3, %3, %4, %8\n\t"
				     "v_alignbit_b32 %4, %4, %5, %8\n\tv_alignbit_b32 %5, %5, %6, %8\n\t"
				     "v_alignbit_b32 %6, %6, %7, %8\n\tv_alignbit_b32 %7, %7, %0, %8"
				     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
				     : "v"(k));
		}
	} else if (OP == 6) {
		uint64_t b0 = a0, b1 = a1, b2 = a2, b3 = a3;
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_lshlrev_b64 %0, %4, %0\n\tv_lshlrev_b64 %1, %4, %1\n\t"
				     "v_lshlrev_b64 %2, %4, %2\n\tv_lshlrev_b64 %3, %4, %3\n\t"
				     "v_lshlrev_b64 %0, %4, %0\n\tv_lshlrev_b64 %1, %4, %1\n\t"
				     "v_lshlrev_b64 %2, %4, %2\n\tv_lshlrev_b64 %3, %4, %3"
				     : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3)
				     : "v"(k));
		}
		a0 = (uint32_t)(b0 ^ b1 ^ b2 ^ b3);
	} else if (OP == 7) {
		float f0 = a0, f1 = a1, f2 = a2, f3 = a3, f4 = a4, f5 = a5, f6 = a6, f7 = a7, fk = (float)k * 1e-9f;
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_fma_f32 %0, %0, %8, %8\n\tv_fma_f32 %1, %1, %8, %8\n\t"
				     "v_fma_f32 %2, %2, %8, %8\n\tv_fma_f32 %3, %3, %8, %8\n\t"
				     "v_fma_f32 %4, %4, %8, %8\n\tv_fma_f32 %5, %5, %8, %8\n\t"
				     "v_fma_f32 %6, %6, %8, %8\n\tv_fma_f32 %7, %7, %8, %8"
				     : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7)
				     : "v"(fk));
		}
		a0 = (uint32_t)(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7);
	} else if (OP == 8) {
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_perm_b32 %0, %0, %1, %8\n\tv_perm_b32 %1, %1, %2, %8\n\t"
				     "v_perm_b32 %2, %2, %3, %8\n\tv_perm_b32 %3, %3, %4, %8\n\t"
				     "v_perm_b32 %4, %4, %5, %8\n\tv_perm_b32 %5, %5, %6, %8\n\t"
				     "v_perm_b32 %6, %6, %7, %8\n\tv_perm_b32 %7, %7, %0, %8"
				     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
				     : "v"(k));
		}
	} else if (OP == 9) { // VOP2 with a literal (8-byte encoding)
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_and_b32 %0, 0x12345, %0\n\tv_and_b32 %1, 0x12345, %1\n\tv_and_b32 %2, 0x12345, %2\n\t"
				     "v_and_b32 %3, 0x12345, %3\n\tv_and_b32 %4, 0x12345, %4\n\tv_and_b32 %5, 0x12345, %5\n\t"
				     "v_and_b32 %6, 0x12345, %6\n\tv_and_b32 %7, 0x12345, %7"
				     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
		}
	} else if (OP == 10) { // VOP2 SDWA
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_add_u32_sdwa %0, %0, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"
				     "v_add_u32_sdwa %1, %1, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"
				     "v_add_u32_sdwa %2, %2, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"
				     "v_add_u32_sdwa %3, %3, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"
				     "v_add_u32_sdwa %4, %4, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"
				     "v_add_u32_sdwa %5, %5, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"
				     "v_add_u32_sdwa %6, %6, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"
				     "v_add_u32_sdwa %7, %7, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD"
				     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
				     : "v"(k));
		}
	} else if (OP == 11) { // VOP3 form of a VOP2 op (v_add_u32_e64)
		CHAINS("v_add_u32_e64")
	} else if (OP == 12) { // VOP3 3-input
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_add3_u32 %0, %0, %8, %1\n\tv_add3_u32 %1, %1, %8, %2\n\tv_add3_u32 %2, %2, %8, %3\n\t"
				     "v_add3_u32 %3, %3, %8, %4\n\tv_add3_u32 %4, %4, %8, %5\n\tv_add3_u32 %5, %5, %8, %6\n\t"
				     "v_add3_u32 %6, %6, %8, %7\n\tv_add3_u32 %7, %7, %8, %0"
				     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
				     : "v"(k));
		}
	} else if (OP == 13) { // VOP2 shifts e32
		CHAINS("v_lshlrev_b32_e32")
	} else if (OP == 14) { // mixed: 1 VOP3 : 1 VOP2
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_alignbit_b32 %0, %0, %1, %8\n\tv_add_u32 %1, %1, %8\n\tv_alignbit_b32 %2, %2, %3, %8\n\t"
				     "v_add_u32 %3, %3, %8\n\tv_alignbit_b32 %4, %4, %5, %8\n\tv_add_u32 %5, %5, %8\n\t"
				     "v_alignbit_b32 %6, %6, %7, %8\n\tv_add_u32 %7, %7, %8"
				     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
				     : "v"(k));
		}
	} else if (OP == 15) { // DPP row_shr:1 (8-byte encoding)
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_add_u32_dpp %0, %0, %8 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
				     "v_add_u32_dpp %1, %1, %8 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
				     "v_add_u32_dpp %2, %2, %8 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
				     "v_add_u32_dpp %3, %3, %8 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
				     "v_add_u32_dpp %4, %4, %8 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
				     "v_add_u32_dpp %5, %5, %8 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
				     "v_add_u32_dpp %6, %6, %8 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
				     "v_add_u32_dpp %7, %7, %8 row_shr:1 row_mask:0xf bank_mask:0xf"
				     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
				     : "v"(k));
		}
	} else if (OP == 16) { // v_cndmask_b32_e32 (vcc)
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_cndmask_b32_e32 %0, %0, %8, vcc\n\tv_cndmask_b32_e32 %1, %1, %8, vcc\n\t"
				     "v_cndmask_b32_e32 %2, %2, %8, vcc\n\tv_cndmask_b32_e32 %3, %3, %8, vcc\n\t"
				     "v_cndmask_b32_e32 %4, %4, %8, vcc\n\tv_cndmask_b32_e32 %5, %5, %8, vcc\n\t"
				     "v_cndmask_b32_e32 %6, %6, %8, vcc\n\tv_cndmask_b32_e32 %7, %7, %8, vcc"
				     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
				     : "v"(k) : "vcc");
		}
	} else if (OP == 17) { // v_cmp (vcc) + v_cndmask_e32 pairs
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_cmp_gt_u32_e32 vcc, %0, %8\n\tv_cndmask_b32_e32 %1, %1, %8, vcc\n\t"
				     "v_cmp_gt_u32_e32 vcc, %2, %8\n\tv_cndmask_b32_e32 %3, %3, %8, vcc\n\t"
				     "v_cmp_gt_u32_e32 vcc, %4, %8\n\tv_cndmask_b32_e32 %5, %5, %8, vcc\n\t"
				     "v_cmp_gt_u32_e32 vcc, %6, %8\n\tv_cndmask_b32_e32 %7, %7, %8, vcc"
				     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
				     : "v"(k) : "vcc");
		}
	} else if (OP == 18) { // v_cndmask_e64 with SGPR mask written once
		uint64_t msk;
		asm volatile("v_cmp_gt_u32_e64 %0, %1, %2" : "=s"(msk) : "v"(a0), "v"(k));
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_cndmask_b32_e64 %0, %0, %8, %9\n\tv_cndmask_b32_e64 %1, %1, %8, %9\n\t"
				     "v_cndmask_b32_e64 %2, %2, %8, %9\n\tv_cndmask_b32_e64 %3, %3, %8, %9\n\t"
				     "v_cndmask_b32_e64 %4, %4, %8, %9\n\tv_cndmask_b32_e64 %5, %5, %8, %9\n\t"
				     "v_cndmask_b32_e64 %6, %6, %8, %9\n\tv_cndmask_b32_e64 %7, %7, %8, %9"
				     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
				     : "v"(k), "s"(msk));
		}
	} else if (OP == 19) {
		CHAINS("v_min_u32")
	} else if (OP == 20) {
		CHAINS("v_sub_u32")
	} else if (OP == 21) {
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_lshl_add_u32 %0, %0, 2, %8\n\tv_lshl_add_u32 %1, %1, 2, %8\n\tv_lshl_add_u32 %2, %2, 2, %8\n\t"
				     "v_lshl_add_u32 %3, %3, 2, %8\n\tv_lshl_add_u32 %4, %4, 2, %8\n\tv_lshl_add_u32 %5, %5, 2, %8\n\t"
				     "v_lshl_add_u32 %6, %6, 2, %8\n\tv_lshl_add_u32 %7, %7, 2, %8"
				     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
				     : "v"(k));
		}
	} else if (OP == 22) {
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_and_or_b32 %0, %0, %8, %1\n\tv_and_or_b32 %1, %1, %8, %2\n\tv_and_or_b32 %2, %2, %8, %3\n\t"
				     "v_and_or_b32 %3, %3, %8, %4\n\tv_and_or_b32 %4, %4, %8, %5\n\tv_and_or_b32 %5, %5, %8, %6\n\t"
				     "v_and_or_b32 %6, %6, %8, %7\n\tv_and_or_b32 %7, %7, %8, %0"
				     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
				     : "v"(k));
		}
	} else if (OP == 23) {
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_bfe_u32 %0, %0, 5, %8\n\tv_bfe_u32 %1, %1, 5, %8\n\tv_bfe_u32 %2, %2, 5, %8\n\t"
				     "v_bfe_u32 %3, %3, 5, %8\n\tv_bfe_u32 %4, %4, 5, %8\n\tv_bfe_u32 %5, %5, 5, %8\n\t"
				     "v_bfe_u32 %6, %6, 5, %8\n\tv_bfe_u32 %7, %7, 5, %8"
				     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
				     : "v"(k));
		}
	} else if (OP == 24) {
		CHAINS("v_mul_u32_u24")
	} else if (OP == 25) {
		CHAINS("v_lshrrev_b32")
	} else if (OP == 26) {
		CHAINS("v_or_b32")
	} else if (OP == 27) {
		CHAINS("v_max_u32")
	} else if (OP == 28) { // lshlrev: varying value, constant shift
		CHAINS("v_lshlrev_b32")
	} else if (OP == 29) {
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_lshlrev_b32 %0, %8, %0\n\tv_lshlrev_b32 %1, %8, %1\n\tv_lshlrev_b32 %2, %8, %2\n\t"
				     "v_lshlrev_b32 %3, %8, %3\n\tv_lshlrev_b32 %4, %8, %4\n\tv_lshlrev_b32 %5, %8, %5\n\t"
				     "v_lshlrev_b32 %6, %8, %6\n\tv_lshlrev_b32 %7, %8, %7"
				     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
				     : "v"(k));
		}
	} else if (OP == 30) {
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_lshrrev_b32 %0, %8, %0\n\tv_lshrrev_b32 %1, %8, %1\n\tv_lshrrev_b32 %2, %8, %2\n\t"
				     "v_lshrrev_b32 %3, %8, %3\n\tv_lshrrev_b32 %4, %8, %4\n\tv_lshrrev_b32 %5, %8, %5\n\t"
				     "v_lshrrev_b32 %6, %8, %6\n\tv_lshrrev_b32 %7, %8, %7"
				     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
				     : "v"(k));
		}
	} else if (OP == 31) {
		CHAINS("v_ashrrev_i32")
	} else if (OP == 32) { // VOPC compare to vcc (8 of them, results unused)
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_cmp_gt_u32_e32 vcc, %0, %8\n\tv_cmp_gt_u32_e32 vcc, %1, %8\n\tv_cmp_gt_u32_e32 vcc, %2, %8\n\t"
				     "v_cmp_gt_u32_e32 vcc, %3, %8\n\tv_cmp_gt_u32_e32 vcc, %4, %8\n\tv_cmp_gt_u32_e32 vcc, %5, %8\n\t"
				     "v_cmp_gt_u32_e32 vcc, %6, %8\n\tv_cmp_gt_u32_e32 vcc, %7, %8"
				     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
				     : "v"(k) : "vcc");
		}
	} else if (OP == 33) {
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_not_b32 %0, %0\n\tv_not_b32 %1, %1\n\tv_not_b32 %2, %2\n\tv_not_b32 %3, %3\n\t"
				     "v_not_b32 %4, %4\n\tv_not_b32 %5, %5\n\tv_not_b32 %6, %6\n\tv_not_b32 %7, %7"
				     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
		}
	} else if (OP == 34) {
		for (int i = 0; i < ITER; i++) {
			asm volatile("v_lshl_or_b32 %0, %0, 2, %8\n\tv_lshl_or_b32 %1, %1, 2, %8\n\tv_lshl_or_b32 %2, %2, 2, %8\n\t"
				     "v_lshl_or_b32 %3, %3, 2, %8\n\tv_lshl_or_b32 %4, %4, 2, %8\n\tv_lshl_or_b32 %5, %5, 2, %8\n\t"
				     "v_lshl_or_b32 %6, %6, 2, %8\n\tv_lshl_or_b32 %7, %7, 2, %8"
				     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
				     : "v"(k));
		}
	} else if (OP == 35) {
		CHAINS("v_subrev_u32")
	} else if (OP == 36) { // v_addc / carry
		{}
	}
	out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

static const char *names[] = {"v_add_u32", "v_xor_b32", "v_pk_add_u16", "v_bfm_b32", "(skip)",
			      "v_alignbit_b32", "v_lshlrev_b64", "v_fma_f32", "v_perm_b32", "v_and_b32+literal",
			      "v_add_u32_sdwa", "v_add_u32_e64", "v_add3_u32", "v_lshlrev_b32_e32", "alignbit:add 1:1",
			      "v_add_u32_dpp", "v_cndmask_b32_e32", "cmp+cndmask (per instr)", "v_cndmask_e64 sgpr",
			      "v_min_u32", "v_sub_u32", "v_lshl_add_u32", "v_and_or_b32", "v_bfe_u32", "v_mul_u32_u24",
			      "v_lshrrev_b32", "v_or_b32", "v_max_u32", "v_lshlrev_b32 (amt varies)", "v_lshlrev_b32 (value varies)",
			      "v_lshrrev_b32 (value varies)", "v_ashrrev_i32", "v_cmp_gt_u32_e32", "v_not_b32", "v_lshl_or_b32",
			      "v_subrev_u32", "(none)"};

template <int OP>
static void run(int cus, int clock_khz, int wps, uint32_t *out)
{
	// 256-thread blocks = 4 waves = one per SIMD; wps blocks per CU
	const int blocks = cus * wps;
	hipEvent_t e0, e1;
	hipEventCreate(&e0);
	hipEventCreate(&e1);
	hipLaunchKernelGGL(bench<OP>, dim3(blocks), dim3(256), 0, 0, out, 3u);
	hipEventRecord(e0, 0);
	hipLaunchKernelGGL(bench<OP>, dim3(blocks), dim3(256), 0, 0, out, 3u);
	hipEventRecord(e1, 0);
	hipEventSynchronize(e1);
	float ms = 0;
	hipEventElapsedTime(&ms, e0, e1);
	const double instr_per_simd = (double)wps * ITER * 8; // wave-instructions per SIMD
	const double cycles = ms * 1e-3 * clock_khz * 1e3;
	printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"cyc_per_instr_per_simd\": %.3f}\n", names[OP],
	       wps, ms, cycles / instr_per_simd);
	hipEventDestroy(e0);
	hipEventDestroy(e1);
}

int main()
{
	int dev = 0, cus = 0, clk = 0;
	hipGetDevice(&dev);
	hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
	hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
	printf("{\"cus\": %d, \"clock_khz\": %d}\n", cus, clk);
	uint32_t *out;
	hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
	for (int wps = 4; wps <= 8; wps *= 2) {
		run<0>(cus, clk, wps, out);
		run<28>(cus, clk, wps, out);
		run<29>(cus, clk, wps, out);
		run<30>(cus, clk, wps, out);
		run<31>(cus, clk, wps, out);
		run<32>(cus, clk, wps, out);
		run<33>(cus, clk, wps, out);
		run<34>(cus, clk, wps, out);
		run<35>(cus, clk, wps, out);
		run<13>(cus, clk, wps, out);
		run<25>(cus, clk, wps, out);
	}
	hipFree(out);
	return 0;
}
