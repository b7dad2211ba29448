// enc_arena.hip -- the arena encode kernel (gfx950): the Rice/ZERO fast path
// of the encode hot loop for 16-bit input.
//
// Same per-sample work as encode_kernel (enc_kernel.h), reference
// lib/compress/cmp.c:296-312: NONE/DIFF residual (preprocess.c:268-300),
// ZigZag (encoder.c:274-286), Golomb ZERO with g = 2^k (encoder.c:327-351,
// zero escape :340-346), big-endian bit packing (bitstream_writer.h:124-158),
// flush (:205-227), header (header.c:24-67).  Eligible: launches with 16-bit
// samples, NONE or DIFF, GOLOMB_ZERO with a power-of-two g <= 2048, no model,
// whole 16 Ki-sample segments and 16-byte aligned frames (cfg2, cfg3, cfg4).
//
// AN EXPERIMENT, OFF BY DEFAULT (AIRS_ARENA=1 turns it on): measured on MI355X
// it is 4-14 % slower than encode_kernel on cfg2, cfg3 and cfg4 in every form
// below (the recomputed table offsets cost more VALU time than
// the barriers and LDS it saves).  Kept bit-exact and tested (test_gpu_arena).
//
// What differs from encode_kernel is where a segment's bits wait for its
// frame offset.  encode_kernel packs chunk by chunk into three rotating chunk
// images sized for the longest codeword (22 bits per sample at k = 5:
// 34 KiB of LDS per workgroup) and must store chunks 0-2 before chunk 3 can
// reuse an image.  Here the segment's exact bit total A is known after the
// lengths pass, so the whole segment is packed back to back into ONE arena
// sized for a typical segment (a launch parameter, ~13 bits per sample):
//   * no image rotation: one barrier before and one after packing all four
//     chunks (encode_kernel: seven), and the look-back is evaluated once the
//     whole segment is packed, so its round trip overlaps all of the packing;
//   * ~25 KiB of LDS and no kept table offsets (the codeword table offsets are
//     recomputed in the packer from the mapped values), so more workgroups
//     fit a CU while a segment waits for its loads or its look-back.
// A segment whose A does not fit the arena (incompressible data) takes four
// passes of one chunk each (any chunk fits: 4096 x 28 bits at k = 11), with
// the look-back after the first.
//
// Look-back, granules, dispatch order and deadlock freedom are those of
// encode_kernel: frame-interleaved segments, one granule
// window of 64 aggregates per round, the first round through scalar loads for
// segments with at least 16 predecessors in their frame, bounded spins.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "enc_common.h"

namespace airs {

#define ACH 4u                     // chunks per segment (= seg_chunks(2, 0))
#define ASEGN (ACH * AIRS_SEG)     // samples per segment
#ifndef AIRS_ARENA_WPE             // minimum waves per SIMD the register allocation must allow
#define AIRS_ARENA_WPE 5
#endif
#ifndef AIRS_ARENA_SLB_N           // granules of the scalar first look-back round
#define AIRS_ARENA_SLB_N 16u
#endif
#ifndef AIRS_PRIO_ARENA            // phase-2 issue priority (encode_kernel AIRS_PRIO_P2)
#define AIRS_PRIO_ARENA 1
#endif
#ifndef AIRS_ARENA_DEFAULT         // eligible launches take the arena kernel (measured slower: off)
#define AIRS_ARENA_DEFAULT 0
#endif
#ifndef AIRS_ARENA_CTL_DEFAULT     // the control-wave form (arena_kernel CTL)
#define AIRS_ARENA_CTL_DEFAULT 0
#endif
#ifndef AIRS_ARENA_AUTO_DEFAULT    // AUTO launches take the arena kernel (with AIRS_ARENA)
#define AIRS_ARENA_AUTO_DEFAULT 1
#endif
#ifndef AIRS_ARENA_KEEPQ
#define AIRS_ARENA_KEEPQ 0
#endif
#ifndef AIRS_ARENA_WORDS_DEFAULT   // arena words: 6400 = 12.5 bits per sample, ~25 KiB of LDS
#define AIRS_ARENA_WORDS_DEFAULT 6400u
#endif

// q = (m + 1) >> k of a pair of mapped values, packed.  v = m + 1 is formed
// with a saturating add, so m = 65535 gives v = 65535 instead of 65536; below
// k = 12 the clamps min(q, 16) / min(q, 17) hide that (q >= 31), from k = 12
// on (AUTO frames only) the lost carry is added back: (65536 >> k) =
// (65535 >> k) + 1 for every k >= 0.
__device__ __forceinline__ u16x2 rice_q(uint32_t mpair, uint32_t k, bool big)
{
	const u16x2 vs = __builtin_elementwise_add_sat(pk(mpair), (u16x2)(1));
	u16x2 q = vs >> (u16x2)((unsigned short)k);
	if (big) {
		const u16x2 vw = pk(mpair) + (u16x2)(1); // wraps to 0 for m = 65535
		q += (vs - vw) >> (u16x2)(15);
	}
	return q;
}

// rice_table_entry (enc_common.h) for every k <= 15: T'[q] mod 2^32, so that
// m + T'[q] is the codeword for q + k + 1 up to 32 bits (q <= 16 at k >= 12,
// so the escape entry 17 is only reached for k <= 11)
__device__ __forceinline__ uint2 rice_entry_any_k(uint32_t q, uint32_t k)
{
	if (q >= 17u)
		return make_uint2(0u, k + 17u);
	const uint64_t t = (1ull << (q + k + 1u)) - (2ull << k) - ((uint64_t)q << k) + 1ull;
	return make_uint2((uint32_t)t, k + 1u + q);
}

// CTL: a fifth wave (the control wave) owns the look-back: it issues the
// scalar granule loads before the packing starts (its barrier instruction
// inside the same asm statement, so that nothing waits for them) and has the
// frame offset in LDS by the barrier that ends the packing; the four data
// waves never wait for the round trip.  Without CTL, wave 0 evaluates the
// look-back after the packing.
//
// AUTO (CMP_GPU_AUTO_RICE, cfg3): the frame's Rice k is chosen from the
// samples already in registers, as encode_kernel's fused selection does
// (DESIGN.md 3.1.1): a 129-bin histogram of (floor(log2 v), next 3 bits) per
// segment in the arena, the 16 candidate sums published as granules, the
// frame's argmin; the same granules give each segment its exact frame offset,
// so there is no look-back, only the predecessor's tail.
template <int PRE, bool STREAM, bool CTL, bool AUTO>
__global__ __launch_bounds__(EWG + (CTL ? 64 : 0)) __attribute__((amdgpu_waves_per_eu(AIRS_ARENA_WPE, 8))) void
arena_kernel(KArgs a)
{
	static_assert(!AUTO || (!CTL && !STREAM), "AUTO: frames, no control wave");
	static_assert(EPT == 16u, "lane t owns samples [16t, 16t+16) of a chunk");
	constexpr uint32_t HDR_BITS = STREAM ? 0u : 176u; // 22-byte header (GOLOMB_ZERO)
	constexpr uint32_t SLB_N = AIRS_ARENA_SLB_N;
	// the arena (a.img_words words, a multiple of 4) after 4 guard words: the
	// packer's first put of a lane ORs zeros into the word before its run
	extern __shared__ __attribute__((aligned(16))) uint32_t L_dyn[];
	uint32_t *const AR = L_dyn + 4u;
	__shared__ uint32_t s_wsum[ACH][EWG / 64];
	__shared__ uint32_t s_misc[4];
	// Rice/ZERO code table: entry min(q, 17) = {T'[q], k + 1 + min(q, 16)},
	// codeword = m + T'[q] (enc_common.h rice_table_entry)
	__shared__ __attribute__((aligned(16))) uint2 s_rice[20];

	const uint32_t tid = threadIdx.x, lane = tid & 63u;
	const uint32_t wid = __builtin_amdgcn_readfirstlane(tid >> 6);
	const bool ctl = CTL && wid == EWG / 64; // the control wave
	const bool data = !ctl;
	const uint32_t lbw = CTL ? EWG / 64 : 0u; // the wave that runs the look-back
	// frame-interleaved dispatch (encode_kernel): consecutive blocks take the
	// same segment index of consecutive frames.  AUTO: frame-major and
	// XCD-local instead (frame 8 j + x takes blocks x + 8 (j spf + s)), so a
	// frame's segments, which wait for each other's candidates, are dispatched
	// together on one XCD; the grid is padded to whole groups of 8 frames
	const uint32_t seg = blockIdx.x;
	const uint32_t nfr = a.num_segs / a.segs_per_frame;
	uint32_t sif, lf;
	if (AUTO) {
		const uint32_t pq = seg >> 3;
		sif = pq % a.segs_per_frame;
		lf = 8u * (pq / a.segs_per_frame) + (seg & 7u);
		if (lf >= nfr)
			return; // padding block
	} else {
		sif = seg / nfr;
		lf = seg - sif * nfr;
	}
	const uint32_t gseg = lf * a.segs_per_frame + sif;
	const uint32_t frame =
		__builtin_amdgcn_readfirstlane(a.frame_list ? a.frame_list[lf] : a.frame_add + lf * a.frame_mul);
	if (frame == AIRS_NO_FRAME)
		return;
	const bool is_first = sif == 0u;
	const bool is_last = sif + 1u == a.segs_per_frame;
	const uint32_t n = a.n;
	const uint8_t *fsrc = a.src + (uint64_t)frame * a.src_stride;

	// ---- phase 0: every load of the segment (32 KiB) up front --------------
	uint4 raw[ACH][2];
	uint32_t prevld[ACH];
#pragma unroll
	for (uint32_t c = 0; c < ACH && data; c++) {
		const uint32_t first = sif * ASEGN + c * AIRS_SEG + tid * EPT;
		const uint4 *p = reinterpret_cast<const uint4 *>(fsrc + (size_t)first * 2u);
		raw[c][0] = p[0];
		raw[c][1] = p[1];
		prevld[c] = 0u;
		if (PRE == PRE_DIFF && lane == 0u && first != 0u)
			prevld[c] = reinterpret_cast<const uint16_t *>(fsrc)[first - 1u];
	}

	// (AUTO: set once the frame's k is chosen)
	uint32_t g = AUTO ? 1u : __builtin_amdgcn_readfirstlane(a.frame_g ? a.frame_g[frame] : a.g);
	Coder cd = make_coder<ENC_ZERO>(g, a.outlier_param);
	uint32_t k = cd.k;
	bool big = false; // k >= 12 (AUTO only): rice_q's exact carry
	if (!AUTO && tid < 18u)
		s_rice[tid] = rice_table_entry(tid, k);

	// ---- phase 1: residuals, mapped values, code lengths (packed 16-bit) ---
	uint32_t mp[ACH][EPT / 2]; // mapped values, two per register
	// AIRS_ARENA_KEEPQ (experiment): the table offsets 8 min(q, 17) kept from
	// the lengths pass (encode_kernel AIRS_KEEP_Q) instead of recomputed
	constexpr bool KQ = AIRS_ARENA_KEEPQ != 0;
	uint32_t mq[KQ ? ACH : 1][EPT / 2];
	uint32_t T[ACH];           // this lane's bits in chunk c
#pragma unroll
	for (uint32_t c = 0; c < ACH; c++) {
		T[c] = 0u;
		if (!data)
			continue;
		uint32_t w[EPT / 2];
#pragma unroll
		for (uint32_t q = 0; q < 2u; q++) {
			w[4 * q] = raw[c][q].x;
			w[4 * q + 1] = raw[c][q].y;
			w[4 * q + 2] = raw[c][q].z;
			w[4 * q + 3] = raw[c][q].w;
		}
		uint32_t wprev = 0u;
		if (PRE == PRE_DIFF) {
			wprev = __shfl_up(w[EPT / 2 - 1], 1, 64);
			if (lane == 0u)
				wprev = prevld[c] << 16;
		}
		u16x2 acc = (u16x2)(0);
#pragma unroll
		for (uint32_t j = 0; j < EPT / 2; j++) {
			uint32_t u = w[j];
			if (PRE == PRE_DIFF)
				u = unpk(pk(w[j]) - pk(__builtin_amdgcn_alignbit(w[j], j ? w[j - 1] : wprev, 16)));
			mp[c][j] = zigzag_pk(u);
			if (!AUTO) {
				const u16x2 q = rice_q(mp[c][j], k, false);
				acc += __builtin_elementwise_min(q, (u16x2)(16));
				if (KQ)
					mq[KQ ? c : 0][j] = unpk(__builtin_elementwise_min(q, (u16x2)(17)) << (u16x2)(3));
			}
		}
		T[c] = EPT * (k + 1u) + (unpk(acc) & 0xFFFFu) + (unpk(acc) >> 16);
		// opaque: the packer recomputes from mp, not from phase 1's temporaries
#pragma unroll
		for (uint32_t i = 0; i < EPT / 2; i++) {
			asm volatile("" : "+v"(mp[c][i]));
			if (KQ)
				asm volatile("" : "+v"(mq[KQ ? c : 0][i]));
		}
	}

	uint32_t auto_P = 0u; // AUTO: the segment's frame bit offset (header included)
	if constexpr (AUTO) {
		// ---- the frame's Rice k ---------------------------
		// 1. histogram: one 32-bit counter per (bin, lane mod 32) in the arena;
		// lanes l and l + 32 share a counter but sit in different LDS lane
		// groups, so the atomics (no return) are conflict-free
		__shared__ uint32_t s_hist[AUTO_BINS];
		__shared__ uint32_t s_kt[EWG / 64][16];
		uint32_t *const H = AR;
		{
			uint4 *Z = reinterpret_cast<uint4 *>(H);
			for (uint32_t i = tid; i < AUTO_BINS * 32u / 4u; i += EWG)
				Z[i] = make_uint4(0u, 0u, 0u, 0u);
		}
		// this lane's counter of bin b is at byte hbase + 128 (b + 1016)
		const uint32_t hbase = (uint32_t)(uintptr_t)H + 4u * (lane & 31u) - 1016u * 128u;
		__syncthreads();
#pragma unroll
		for (uint32_t c = 0; c < ACH; c++) {
#pragma unroll
			for (uint32_t jp = 0; jp < EPT / 2; jp++) {
				// an opaque copy: otherwise the bins are computed ahead of the
				// barrier above (~150 more VGPRs)
				uint32_t wv = mp[c][jp];
				asm volatile("" : "+v"(wv));
#pragma unroll
				for (uint32_t h = 0; h < 2; h++) {
					const uint32_t v = half16(wv, h) + 1u;
					// bin + 1016 = the top 12 bits of the float v
					uint32_t ha;
					asm("v_lshrrev_b32 %0, 20, %1\n\tv_lshl_add_u32 %0, %0, 7, %2"
					    : "=&v"(ha)
					    : "v"(__float_as_uint((float)v)), "v"(hbase));
					__hip_atomic_fetch_add(reinterpret_cast<lds_u32 *>((uintptr_t)ha), 1u, __ATOMIC_RELAXED,
							       __HIP_MEMORY_SCOPE_WORKGROUP);
				}
			}
		}
		__syncthreads();
		// 2. bin totals: threads 2r, 2r + 1 sum the halves of row r < 128
		// (four 16-byte reads each); wave 0 sums row 128 (v = 65536)
		{
			const uint32_t r = tid >> 1, hh = tid & 1u;
			const uint4 *row = reinterpret_cast<const uint4 *>(H + r * 32u + hh * 16u);
			uint32_t sm = 0u;
#pragma unroll
			for (uint32_t q = 0; q < 4u; q++) {
				const uint4 x = row[(q + r) & 3u];
				sm += x.x + x.y + x.z + x.w;
			}
			sm += __shfl_xor(sm, 1, 64);
			if (hh == 0u)
				s_hist[r] = sm;
			static_assert(AUTO_BINS == EWG / 2u + 1u, "rows 0..127 by thread pairs, then row 128");
			if (wid == 0) {
				const uint32_t s128 = wave_sum(lane < 32u ? H[128u * 32u + lane] : 0u);
				if (lane == 0)
					s_hist[128] = s128;
			}
		}
		__syncthreads();
		// 3. this segment's 16 candidate sums: thread (slice sl, k) covers
		// bins sl, sl + 16, ...; the four slices of a wave meet by shuffles
		{
			const uint32_t kk = tid & 15u, sl = tid >> 4;
			uint32_t part = 0u;
#pragma unroll
			for (uint32_t i = 0; i < (AUTO_BINS + 15u) / 16u; i++) {
				const uint32_t b = sl + 16u * i;
				if (b < AUTO_BINS) {
					// min(v >> kk, 16) of every v in bin b (encode_kernel auto_term)
					const uint32_t t = b >> 3, top4 = 8u + (b & 7u);
					const uint32_t term = kk + 4u <= t ? 16u : kk > t ? 0u : top4 >> (kk + 3u - t);
					part += s_hist[b] * term;
				}
			}
			part += __shfl_xor(part, 16, 64);
			part += __shfl_xor(part, 32, 64);
			if (lane < 16u)
				s_kt[wid][kk] = part;
		}
		__syncthreads();
		if (wid == 0) {
			// 4. publish (lanes 0-15), then read the frame's 16 spf granules
			if (lane < 16u) {
				const uint32_t sk = s_kt[0][lane] + s_kt[1][lane] + s_kt[2][lane] + s_kt[3][lane];
				gran_store(&a.ktot[(uint64_t)gseg * 16u + lane], ((uint64_t)a.epoch << 32) | sk);
			}
			const uint32_t fs = gseg - sif, ng = a.segs_per_frame * 16u;
			constexpr uint32_t NL = (AUTO_MAX_SPF + 3u) / 4u; // granule loads per lane
			uint64_t gk[NL];
#pragma unroll
			for (uint32_t i = 0; i < NL; i++) {
				const uint32_t gi = 64u * i + lane;
				gk[i] = gran_load(&a.ktot[(uint64_t)fs * 16u + (gi < ng ? gi : 0u)]);
			}
			for (uint32_t spins = 0;;) {
				bool bad = false;
#pragma unroll
				for (uint32_t i = 0; i < NL; i++)
					bad |= 64u * i + lane < ng && (uint32_t)(gk[i] >> 32) != a.epoch;
				if (!__ballot(bad))
					break;
				if (++spins > AIRS_SPIN_LIMIT) {
					if (lane == 0)
						atomicAdd(a.ticket + AIRS_FAULT_WORD, 1u);
					break;
				}
				__builtin_amdgcn_s_sleep(1);
#pragma unroll
				for (uint32_t i = 0; i < NL; i++) {
					const uint32_t gi = 64u * i + lane;
					if (gi < ng && (uint32_t)(gk[i] >> 32) != a.epoch)
						gk[i] = gran_load(&a.ktot[(uint64_t)fs * 16u + gi]);
				}
			}
			// lane l holds segment 4 i + l / 16, candidate k = l % 16
			uint32_t tot = 0u, pre = 0u;
#pragma unroll
			for (uint32_t i = 0; i < NL; i++) {
				const uint32_t gi = 64u * i + lane;
				const uint32_t v = gi < ng ? (uint32_t)gk[i] : 0u;
				tot += v;
				pre += (gi >> 4) < sif ? v : 0u;
			}
			tot += __shfl_xor(tot, 16, 64);
			tot += __shfl_xor(tot, 32, 64);
			pre += __shfl_xor(pre, 16, 64);
			pre += __shfl_xor(pre, 32, 64);
			const uint32_t kk = lane & 15u;
			// frame bits for k (< 2^28: spf <= 32 segments), ties to the smaller k
			uint32_t key = ((tot + n * (kk + 1u)) << 4) | kk;
#pragma unroll
			for (uint32_t d = 1; d < 16u; d <<= 1)
				key = min(key, (uint32_t)__shfl_xor(key, d, 64));
			const uint32_t ks = key & 15u;
			const uint32_t pre_k = __shfl(pre, ks, 64);
			if (lane == 0) {
				s_misc[0] = ks;
				// every segment before this one is whole
				s_misc[3] = HDR_BITS + pre_k + sif * ASEGN * (ks + 1u);
			}
		}
		__syncthreads();
		k = __builtin_amdgcn_readfirstlane(s_misc[0]);
		auto_P = __builtin_amdgcn_readfirstlane(s_misc[3]);
		g = 1u << k;
		cd = make_coder<ENC_ZERO>(g, a.outlier_param);
		big = k >= 12u;
		if (tid < 18u)
			s_rice[tid] = rice_entry_any_k(tid, k);
		// the code lengths, now that k is known
#pragma unroll
		for (uint32_t c = 0; c < ACH; c++) {
			u16x2 acc = (u16x2)(0);
#pragma unroll
			for (uint32_t j = 0; j < EPT / 2; j++) {
				const u16x2 q = rice_q(mp[c][j], k, big);
				acc += __builtin_elementwise_min(q, (u16x2)(16));
				if (KQ)
					mq[KQ ? c : 0][j] = unpk(__builtin_elementwise_min(q, (u16x2)(17)) << (u16x2)(3));
			}
			T[c] = EPT * (k + 1u) + (unpk(acc) & 0xFFFFu) + (unpk(acc) >> 16);
#pragma unroll
			for (uint32_t i = 0; i < EPT / 2; i++) {
				asm volatile("" : "+v"(mp[c][i]));
				if (KQ)
					asm volatile("" : "+v"(mq[KQ ? c : 0][i]));
			}
		}
	}

	// ---- per-chunk block scans (DPP within waves, LDS across waves) -------
	uint32_t inc[ACH];
#pragma unroll
	for (uint32_t c = 0; c < ACH; c++) {
		inc[c] = wave_incl_scan(T[c]);
		if (lane == 63u && data)
			s_wsum[c][wid] = inc[c];
	}
	__syncthreads(); // B1: wave totals and the code table visible
	uint32_t excl[ACH], base[ACH + 1];
	uint32_t A = 0u;
#pragma unroll
	for (uint32_t c = 0; c < ACH; c++) {
		uint32_t woff = 0u, tt = 0u;
#pragma unroll
		for (uint32_t w = 0; w < EWG / 64; w++) {
			const uint32_t v = s_wsum[c][w];
			woff += w < wid ? v : 0u;
			tt += v;
		}
		excl[c] = woff + inc[c] - T[c];
		base[c] = A;
		A += __builtin_amdgcn_readfirstlane(tt);
	}
	base[ACH] = A;
	const uint32_t first_seg = gseg - sif;
	if (!AUTO && wid == lbw && lane == 0) {
		const uint64_t tag = ((uint64_t)a.epoch << 1) | (is_first ? 1u : 0u);
		gran_store(&a.agg[gseg], (tag << 32) | (is_first ? HDR_BITS + A : A));
	}
	const char *tab = reinterpret_cast<const char *>(s_rice);
	if (!is_last && wid == EWG / 64 - 1) {
		// the segment's last 32 bits for the successor's first word (wave 3
		// rebuilds the last chunk's codewords; every sample takes >= k + 1
		// bits, so for k >= 3 a lane's last 32 bits lie in its last 8 samples)
		uint64_t acc = 0u;
#pragma unroll
		for (uint32_t j = 0; j < EPT / 2; j++) {
			if (j < EPT / 4 && k >= 3u)
				continue;
			const uint32_t qa =
				unpk(__builtin_elementwise_min(rice_q(mp[ACH - 1][j], k, big), (u16x2)(17)) << (u16x2)(3));
#pragma unroll
			for (uint32_t h = 0; h < 2; h++) {
				const uint2 e = *reinterpret_cast<const uint2 *>(tab + half16(qa, h));
				acc = (acc << e.y) | (half16(mp[ACH - 1][j], h) + e.x);
			}
		}
		uint32_t v = (uint32_t)acc, tb = min(T[ACH - 1], 32u);
#pragma unroll
		for (uint32_t d = 1; d <= 2; d <<= 1) {
			const uint32_t va = __shfl_up(v, d, 64), ta = __shfl_up(tb, d, 64);
			if (lane >= d && tb < 32u) {
				v = (va << tb) | v;
				tb = min(ta + tb, 32u);
			}
		}
		if (lane == 63u)
			gran_store(&a.tail[gseg], ((uint64_t)a.epoch << 32) | v);
	}

	uint8_t *fdst = a.dst + (uint64_t)frame * a.dst_stride;
	const uint32_t cap = a.cap;
	const __amdgpu_buffer_rsrc_t dst_rsrc = __builtin_amdgcn_make_buffer_rsrc(fdst, 0, (int)(cap & ~3u), 0x00020000);

	// Store an image of `totx` bits at frame bit Pc, funnel-shifted by Pc mod
	// 32 (encode_kernel store_chunk).  Word 0 takes the 32 stream bits before
	// Pc from predx (thread 0).  Complete words only; the last partial word is
	// the successor's word 0, or, for the frame's end, the zero-padded final
	// bytes (reference bitstream_flush).  The buffer range (cap & ~3) drops
	// the words that would not fit.
	auto store_image = [&](uint32_t Pc, uint32_t totx, uint32_t predx, bool finalx) {
		const uint32_t r = Pc & 31u, g0 = Pc >> 5;
		const uint32_t endbit = Pc + totx;
		const uint32_t J = ((endbit - 1u) >> 5) - g0;
		const uint32_t nfull = (endbit & 31u) == 0u ? J + 1u : J;
		const lds_u32 *Ll = reinterpret_cast<const lds_u32 *>((uintptr_t)AR);
		const uint32_t nquad = nfull >> 2;
		for (uint32_t p = tid; p < nquad; p += EWG) {
			const uint32_t j = 4u * p;
			const u32x4 w = *reinterpret_cast<const __attribute__((address_space(3))) u32x4 *>(Ll + j);
			const uint32_t hi = j ? Ll[j - 1u] : predx;
			u32x4 o;
			o.x = bswap32(__builtin_amdgcn_alignbit(hi, w.x, r));
			o.y = bswap32(__builtin_amdgcn_alignbit(w.x, w.y, r));
			o.z = bswap32(__builtin_amdgcn_alignbit(w.y, w.z, r));
			o.w = bswap32(__builtin_amdgcn_alignbit(w.z, w.w, r));
			__builtin_amdgcn_raw_buffer_store_b128(o, dst_rsrc, (int)(4u * (g0 + j)), 0, 0);
		}
		const uint32_t rr = (tid - nquad) & (EWG - 1u);
		if (rr < (nfull & 3u)) {
			const uint32_t j = 4u * nquad + rr;
			const uint32_t hi = j ? Ll[j - 1u] : predx;
			const uint32_t v = __builtin_amdgcn_alignbit(hi, Ll[j], r);
			__builtin_amdgcn_raw_buffer_store_b32(bswap32(v), dst_rsrc, (int)(4u * (g0 + j)), 0, 0);
		}
		if (finalx && nfull == J && tid == 0) {
			const uint32_t hi = J ? AR[J - 1u] : predx;
			const uint32_t v = __builtin_amdgcn_alignbit(hi, AR[J], r);
			const uint32_t gw = g0 + J;
			const uint32_t nbytes = ((endbit & 31u) + 7u) >> 3;
			for (uint32_t b = 0; b < nbytes; b++)
				if (4u * gw + b < cap)
					fdst[4u * gw + b] = (uint8_t)(v >> (24u - 8u * b));
		}
	};

	// ---- the look-back (wave lbw) ---------------------------------------
	// First round: the 64 newest granules through vector loads for segments
	// with fewer than SLB_N predecessors in their frame; else the SLB_N newest
	// (and the predecessor's tail) through scalar loads, which do not queue
	// behind the CU's sample loads.  slb_load issues them and
	// waits in ONE asm statement (lgkmcnt also counts LDS operations, and no
	// register of an outstanding load may be visible to the compiler); with
	// CTL the statement also holds the control wave's barrier B2.
	typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
	auto sptr = [](const uint64_t *p) {
		const uint64_t v = (uint64_t)(uintptr_t)p;
		const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)v);
		const uint32_t h = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
		return (const uint64_t *)(uintptr_t)(((uint64_t)h << 32) | l);
	};
	auto slb_load = [&](uint64_t &gv, uint64_t &tv0, bool with_barrier) {
		const uint64_t *gp = sptr(&a.agg[gseg - SLB_N]);
		const uint64_t *tp = sptr(&a.tail[gseg - 1u]);
		u32x16 q[2];
		uint64_t tq;
		if (with_barrier)
			asm volatile("s_load_dwordx16 %0, %3, 0x0 glc\n\t"
				     "s_load_dwordx16 %1, %3, 0x40 glc\n\t"
				     "s_load_dwordx2 %2, %4, 0x0 glc\n\t"
				     "s_barrier\n\t"
				     "s_waitcnt lgkmcnt(0)"
				     : "=&s"(q[0]), "=&s"(q[1]), "=&s"(tq)
				     : "s"(gp), "s"(tp)
				     : "memory");
		else
			asm volatile("s_load_dwordx16 %0, %3, 0x0 glc\n\t"
				     "s_load_dwordx16 %1, %3, 0x40 glc\n\t"
				     "s_load_dwordx2 %2, %4, 0x0 glc\n\t"
				     "s_waitcnt lgkmcnt(0)"
				     : "=&s"(q[0]), "=&s"(q[1]), "=&s"(tq)
				     : "s"(gp), "s"(tp)
				     : "memory");
		// granule gseg - SLB_N + i -> lane SLB_N - 1 - i; lanes >= SLB_N read as
		// unpublished (tag 0).  (v_writelane: no per-lane compares, which the
		// compiler hoisted and spilled)
		uint32_t vl = 0u, vh = 0u;
#pragma unroll
		for (uint32_t i = 0; i < SLB_N; i++) {
			asm("v_writelane_b32 %0, %1, %2" : "+v"(vl) : "s"(q[i >> 3][2u * (i & 7u)]), "n"(SLB_N - 1u - i));
			asm("v_writelane_b32 %0, %1, %2" : "+v"(vh) : "s"(q[i >> 3][2u * (i & 7u) + 1u]), "n"(SLB_N - 1u - i));
		}
		gv = ((uint64_t)vh << 32) | vl;
		tv0 = tq;
	};
	auto vec_load = [&](uint64_t &gv, uint64_t &tv0) {
		const int64_t idx = (int64_t)gseg - 1 - (int64_t)lane;
		gv = gran_load(&a.agg[idx >= (int64_t)first_seg ? idx : (int64_t)first_seg]);
		tv0 = gran_load(&a.tail[gseg - 1u]);
	};
	// rounds until an inclusive prefix: the frame offset P, published as this
	// segment's inclusive prefix; the predecessor's tail; both to LDS
	auto evaluate = [&](uint64_t gv, uint64_t tv0) {
		uint32_t Pw = HDR_BITS, prd = 0u;
		if (is_first) {
			// header bytes 20-21 (low half of the outlier field) share the
			// first payload dword of the 22-byte header
			prd = STREAM ? 0u : (cd.outlier & 0xFFFFu);
		} else if (AUTO) {
			Pw = auto_P; // from the frame's candidate granules
			if (lane == 0) {
				uint64_t tv = tv0;
				for (uint32_t sp = 0; (uint32_t)(tv >> 32) != a.epoch; sp++) {
					if (sp > AIRS_SPIN_LIMIT) {
						atomicAdd(a.ticket + AIRS_FAULT_WORD, 1u);
						break;
					}
					__builtin_amdgcn_s_sleep(1);
					tv = gran_load(&a.tail[gseg - 1u]);
				}
				prd = (uint32_t)tv;
			}
		} else {
			uint32_t sum = 0u, spins = 0u;
			int64_t j = (int64_t)gseg - 1;
			for (;;) {
				const int64_t idx = j - (int64_t)lane;
				const bool inr = idx >= (int64_t)first_seg;
				const uint32_t tag = (uint32_t)(gv >> 32);
				const bool valid = inr && (tag >> 1) == a.epoch;
				const bool incl = valid && (tag & 1u);
				const uint64_t incl_m = __ballot(incl);
				const uint64_t bad_m = __ballot(inr && !valid);
				const uint32_t fi = incl_m ? (uint32_t)__ffsll((unsigned long long)incl_m) - 1u : 64u;
				const uint64_t need = fi >= 63u ? ~0ull : ((2ull << fi) - 1ull);
				if (bad_m & need) {
					// a needed predecessor has not published: re-poll this window
					if (++spins > AIRS_SPIN_LIMIT) {
						if (lane == 0)
							atomicAdd(a.ticket + AIRS_FAULT_WORD, 1u);
						break;
					}
					__builtin_amdgcn_s_sleep(1);
				} else {
					sum += wave_sum((inr && lane <= fi) ? (uint32_t)gv : 0u);
					if (incl_m)
						break;
					j -= 64;
				}
				const int64_t id2 = j - (int64_t)lane;
				gv = id2 >= (int64_t)first_seg ? gran_load(&a.agg[id2]) : 0ull;
			}
			Pw = sum;
			if (lane == 0)
				gran_store(&a.agg[gseg], ((((uint64_t)a.epoch << 1) | 1u) << 32) | (Pw + A));
			if (lane == 0) {
				uint64_t tv = tv0;
				for (uint32_t sp = 0; (uint32_t)(tv >> 32) != a.epoch; sp++) {
					if (sp > AIRS_SPIN_LIMIT) {
						atomicAdd(a.ticket + AIRS_FAULT_WORD, 1u);
						break;
					}
					__builtin_amdgcn_s_sleep(1);
					tv = gran_load(&a.tail[gseg - 1u]);
				}
				prd = (uint32_t)tv;
			}
		}
		if (lane == 0) {
			s_misc[1] = Pw;
			s_misc[2] = prd;
		}
	};

	// ---- phase 2: passes of whole chunks -> the arena -> HBM ----------------
	// one pass of all four chunks when the segment fits the arena, else one
	// pass per chunk (uniform: A is block-uniform)
	const bool one_pass = A + 64u <= 32u * a.img_words;
	const uint32_t npass = one_pass ? 1u : ACH;
	if (AIRS_PRIO_ARENA)
		__builtin_amdgcn_s_setprio(1);
	uint32_t P = HDR_BITS;     // the segment's frame bit offset (after the look-back)
	uint32_t pred = 0u;        // (thread 0) the 32 stream bits before the pass
	for (uint32_t ps = 0; ps < npass; ps++) {
		const uint32_t c0 = one_pass ? 0u : ps, c1 = one_pass ? ACH : ps + 1u;
		const uint32_t pb0 = one_pass ? 0u : base[ps];
		const uint32_t pbits = one_pass ? A : base[ps + 1u] - base[ps];
		// zero the words this pass touches (the previous pass's stores have
		// read the arena before the barrier that ended its look-back / pass)
		if (ps)
			__syncthreads();
		if (data) {
			uint4 *Z = reinterpret_cast<uint4 *>(AR);
			const uint32_t nz4 = (((pbits + 31u) >> 5) + 4u) >> 2;
			for (uint32_t i = tid; i < nz4; i += EWG)
				Z[i] = make_uint4(0u, 0u, 0u, 0u);
		}
		uint64_t gv = 0, tv0 = 0;
		const bool lb = ps == 0 && !is_first; // this pass runs the look-back
		if (CTL && ctl) {
			// B2 for the control wave, with the first round's loads in flight
			if (lb && sif >= SLB_N) {
				slb_load(gv, tv0, true);
			} else {
				if (lb)
					vec_load(gv, tv0);
				asm volatile("s_barrier" ::: "memory");
			}
		} else {
			__syncthreads(); // B2: arena zeroed
		}
		if (!CTL && lb && AUTO && wid == 0)
			tv0 = gran_load(&a.tail[gseg - 1u]); // AUTO: only the predecessor's tail
		else if (!CTL && lb && sif < SLB_N && wid == 0)
			vec_load(gv, tv0); // issued here, evaluated after the packing
#pragma unroll
		for (uint32_t c = 0; c < ACH; c++) {
			if (c < c0 || c >= c1 || !data)
				continue;
			// opaque per pass: otherwise the table offsets of every chunk are
			// hoisted out of the pass loop (~70 more VGPRs)
#pragma unroll
			for (uint32_t i = 0; i < EPT / 2; i++) {
				asm volatile("" : "+v"(mp[c][i]));
				if (KQ)
					asm volatile("" : "+v"(mq[KQ ? c : 0][i]));
			}
			Packer pk1;
			pk1.init(AR, base[c] - pb0 + excl[c]);
#pragma unroll
			for (uint32_t hb = 0; hb < 2; hb++) { // two batches of 8 lookups
				uint2 te[EPT / 2];
#pragma unroll
				for (uint32_t jj = 0; jj < EPT / 4; jj++) {
					const uint32_t j = hb * (EPT / 4) + jj;
					const uint32_t qa =
						KQ ? mq[KQ ? c : 0][j]
						   : unpk(__builtin_elementwise_min(rice_q(mp[c][j], k, big), (u16x2)(17)) << (u16x2)(3));
#pragma unroll
					for (uint32_t h = 0; h < 2; h++)
						te[2 * jj + h] = *reinterpret_cast<const uint2 *>(tab + half16(qa, h));
				}
				uint32_t mxl = 0u;
#pragma unroll
				for (uint32_t i = 0; i < EPT / 2; i += 2)
					mxl = max(mxl, te[i].y + te[i + 1].y);
				if (__ballot(mxl > 32u) == 0ull) {
#pragma unroll
					for (uint32_t i = 0; i < EPT / 2; i += 2) {
						const uint32_t j = hb * (EPT / 4) + i / 2;
						const uint32_t cwa = (mp[c][j] & 0xFFFFu) + te[i].x;
						const uint32_t cwb = (mp[c][j] >> 16) + te[i + 1].x;
						pk1.put((cwa << te[i + 1].y) | cwb, te[i].y + te[i + 1].y);
					}
				} else {
#pragma unroll
					for (uint32_t i = 0; i < EPT / 2; i += 2) {
						const uint32_t j = hb * (EPT / 4) + i / 2;
						pk1.put((mp[c][j] & 0xFFFFu) + te[i].x, te[i].y);
						pk1.put((mp[c][j] >> 16) + te[i + 1].x, te[i + 1].y);
					}
				}
			}
			pk1.flush();
			// keep the chunks' table lookups apart (hoisted, they cost ~80 VGPRs)
			__builtin_amdgcn_sched_barrier(0);
		}
		if (CTL && ctl && ps == 0)
			evaluate(gv, tv0); // while the data waves pack
		__syncthreads(); // B3: the pass is packed (CTL: and the frame offset is in LDS)
		uint32_t pred_next = 0u; // (thread 0) the pass's last 32 bits, for the next pass
		if (ps + 1u < npass && tid == 0) {
			const uint32_t s0 = pbits - 32u, q = s0 >> 5, sh = s0 & 31u;
			pred_next = sh ? (AR[q] << sh) | (AR[q + 1] >> (32u - sh)) : AR[q];
		}
		if (ps == 0) {
			if (!CTL) {
				// ---- decoupled look-back (wave 0), after the packing --------
				if (wid == 0) {
					if (!AUTO && lb && sif >= SLB_N)
						slb_load(gv, tv0, false);
					evaluate(gv, tv0);
				}
				__syncthreads(); // B4: the frame offset
			}
			P = __builtin_amdgcn_readfirstlane(s_misc[1]);
			pred = s_misc[2];
		}
		if (data)
			store_image(P + pb0, pbits, pred, is_last && c1 == ACH);
		pred = pred_next;
	}

	// ---- frame epilogue: checksum, header, status ------------------------
	if (STREAM && is_last && tid == 0) {
		const uint32_t payload_bytes = (P + A + 7u) >> 3;
		a.status[frame] = payload_bytes > cap ? ERRV(E_DST_TOO_SMALL) : payload_bytes;
		if (a.needed)
			a.needed[frame] = payload_bytes;
	}
	if (!STREAM && is_last && tid == 0) {
		const uint32_t endbit = P + A;
		const uint32_t payload_bytes = (endbit + 7u) >> 3;
		const uint32_t size = payload_bytes + (a.checksum ? 4u : 0u);
		if (a.checksum) {
			const uint32_t ck = a.checksums[frame];
			for (uint32_t b = 0; b < 4u; b++)
				if (payload_bytes + b < cap)
					fdst[payload_bytes + b] = (uint8_t)(ck >> (24u - 8u * b));
		}
		const uint64_t id = a.ids ? a.ids[lf] : a.id_base + (uint64_t)lf * a.id_step;
		uint32_t h[5];
		header_words(h, size, 2u * n, id, a.seqs ? a.seqs[frame] : a.seq, PRE, a.checksum ? 1u : 0u, ENC_ZERO, 0u,
			     g, cd.outlier);
#pragma unroll
		for (uint32_t w = 0; w < 5u; w++)
			if (4u * w + 4u <= cap)
				*reinterpret_cast<uint32_t *>(fdst + 4u * w) = bswap32(h[w]);
		uint32_t st = size;
		if (size > cap)
			st = ERRV(E_DST_TOO_SMALL);
		else if (size > 0xFFFFFFu)
			st = ERRV(E_HDR_CMP_SIZE_TOO_LARGE);
		a.status[frame] = st;
		if (a.needed)
			a.needed[frame] = size;
	}
}

// arena words for a launch: AIRS_ARENA_WORDS (env, experiments) or the
// build default; at least one chunk of 28-bit codewords (k <= 11)
uint32_t arena_words()
{
	static uint32_t w = 0;
	if (!w) {
		uint32_t v = AIRS_ARENA_WORDS_DEFAULT;
		if (const char *s = getenv("AIRS_ARENA_WORDS"))
			v = (uint32_t)atoi(s);
		const uint32_t lo = AIRS_SEG * 28u / 32u + 8u;
		v = v < lo ? lo : v;
		w = (v + 3u) & ~3u;
	}
	return w;
}

// AIRS_ARENA=1 (env, read at every launch: A/B experiments and the arena's
// parity tests) sends the eligible launches to the arena kernel; measured
// slower than encode_kernel on every workload, so off by default
bool arena_enabled()
{
	const char *s = getenv("AIRS_ARENA");
	return s ? atoi(s) != 0 : AIRS_ARENA_DEFAULT != 0;
}

// AIRS_ARENA_CTL (env, A/B experiments): 1 = the control-wave form
static bool arena_ctl()
{
	static int on = -1;
	if (on < 0) {
		const char *s = getenv("AIRS_ARENA_CTL");
		on = s ? atoi(s) != 0 : AIRS_ARENA_CTL_DEFAULT;
	}
	return on != 0;
}

template <int PRE, bool STREAM>
static void arena_go(const KArgs &k, uint32_t grid, size_t lds, hipStream_t s)
{
	if (arena_ctl())
		hipLaunchKernelGGL((arena_kernel<PRE, STREAM, true, false>), dim3(grid), dim3(EWG + 64), lds, s, k);
	else
		hipLaunchKernelGGL((arena_kernel<PRE, STREAM, false, false>), dim3(grid), dim3(EWG), lds, s, k);
}

// AUTO launches (k.ktot set; grid padded to whole groups of 8 frames)
bool arena_auto_encode(const KArgs &k, uint32_t pre, uint32_t grid, hipStream_t s)
{
	const size_t lds = (size_t)(k.img_words + 4u) * 4u;
	if (pre == PRE_DIFF)
		hipLaunchKernelGGL((arena_kernel<PRE_DIFF, false, false, true>), dim3(grid), dim3(EWG), lds, s, k);
	else if (pre == PRE_NONE)
		hipLaunchKernelGGL((arena_kernel<PRE_NONE, false, false, true>), dim3(grid), dim3(EWG), lds, s, k);
	else
		return false;
	return true;
}

// AIRS_ARENA_AUTO=0 (env, A/B experiments) keeps AUTO launches on encode_kernel
bool arena_auto_enabled()
{
	const char *e = getenv("AIRS_ARENA_AUTO");
	return (e ? atoi(e) != 0 : AIRS_ARENA_AUTO_DEFAULT != 0) && arena_enabled();
}

bool arena_encode(const KArgs &k, uint32_t pre, bool stream, uint32_t grid, hipStream_t s)
{
	const size_t lds = (size_t)(k.img_words + 4u) * 4u;
	if (pre == PRE_DIFF) {
		if (stream)
			arena_go<PRE_DIFF, true>(k, grid, lds, s);
		else
			arena_go<PRE_DIFF, false>(k, grid, lds, s);
	} else if (pre == PRE_NONE) {
		if (stream)
			arena_go<PRE_NONE, true>(k, grid, lds, s);
		else
			arena_go<PRE_NONE, false>(k, grid, lds, s);
	} else {
		return false;
	}
	return true;
}

} // namespace airs
