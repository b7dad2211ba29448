// enc_kernel.h -- the encode kernel template (encode_kernel), shared by
// encode.hip (frame launches) and enc_stream.hip (payload-only streams), so
// that its instantiations compile in separate translation units.  Reference
// citations as in encode.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "enc_common.h"

namespace airs {

// ---------------------------------------------------------------------
// the encode kernel
//   W      bytes per input sample (2: u16/i16, 4: i16 in i32)
//   PRE    NONE / DIFF / MODEL
//   ENC    UNCOMPRESSED / GOLOMB_ZERO / GOLOMB_MULTI
//   RICE   Golomb parameter is a power of two (shift instead of divide)
//   MODEL  0: no model, 1: store samples (primary pass), 2: update (secondary)
//
// One workgroup encodes one segment of SEG_CHUNKS(W, MODEL) chunks of 4096
// samples; lane t owns samples [16t, 16t+16) of every chunk.  All chunk loads
// are issued up front (32 KiB per workgroup for u16) so HBM sees many bytes in
// flight per CU.  Phase 1 computes only code lengths, so the segment's bit
// total and its last 32 bits are published early; phase 2 rebuilds the
// codewords chunk by chunk into a double-buffered LDS image and stores them
// once the look-back has produced the segment's frame bit offset.
// ---------------------------------------------------------------------
#ifndef AIRS_SEG_CH
#define AIRS_SEG_CH 4
#endif
#ifndef AIRS_SEG_CH_WIDE // chunks per segment for i16-in-i32 and MODEL launches
#define AIRS_SEG_CH_WIDE 2
#endif
__host__ __device__ constexpr uint32_t seg_chunks(int W, int MODEL)
{
	return (W == 4 || MODEL) ? AIRS_SEG_CH_WIDE : AIRS_SEG_CH;
}
// LDS chunk images per workgroup: with three, the look-back is evaluated
// after the third chunk's packing (chunks 0 and 1 are stored late)
#ifndef AIRS_NIMG
#define AIRS_NIMG 3
#endif
__host__ __device__ constexpr uint32_t seg_images(int W, int MODEL)
{
	return (seg_chunks(W, MODEL) >= 4u && !MODEL) ? AIRS_NIMG : 2u;
}

#ifdef AIRS_EWPE // minimum waves per SIMD the register allocation must allow
#define AIRS_EWPE_ATTR __attribute__((amdgpu_waves_per_eu(AIRS_EWPE, 8)))
#else
#define AIRS_EWPE_ATTR
#endif
// Fused per-frame Rice selection (AUTO, CMP_GPU_AUTO_RICE): the rule is
// k = argmin over k = 0..15 of n(k+1) + sum_i min(v_i >> k, 16), v = m + 1
// (oracle orc_select_rice_k).  The 129-bin histogram of (floor(log2 v), the
// next 3 bits of v) is a sufficient statistic: its bin is the top 11 bits of
// the float v, less 1016.  term(bin, k) is that bin's min(v >> k, 16).
#ifndef AIRS_AUTO_ABLATE // experiments: 1 no histogram atomics, 2 no wait for the frame
#define AIRS_AUTO_ABLATE 0
#endif
#define AIRS_AUTO_ABL(b) ((AIRS_AUTO_ABLATE & (b)) != 0)

template <int W, int PRE, int ENC, bool RICE, int MODEL, bool FULL, bool AUTO = false, bool STREAM = false>
__global__ __launch_bounds__(EWG) AIRS_EWPE_ATTR void encode_kernel(KArgs a)
{
	// AUTO: the frame's k is chosen here from the samples already in registers
	// (one read); the frame's segments meet once at the 16-candidate granules,
	// which also give every segment its exclusive bit offset (no look-back)
	constexpr bool AUTOK = AUTO && ENC == ENC_ZERO && RICE && MODEL == 0 && (PRE == PRE_NONE || PRE == PRE_DIFF);
	constexpr uint32_t CH = seg_chunks(W, MODEL);
	constexpr uint32_t SEGN = CH * AIRS_SEG;
	constexpr uint32_t NPIECE = ENC == ENC_MULTI ? 2 : 1;
	// Chunk after whose packing the look-back is evaluated.  1: wave 0 issues
	// the granule loads when chunk 1's packing starts and reads them when it
	// ends, so they see the predecessors one chunk later than the aggregate
	// publish (which an earlier poll mostly misses); chunk 0 is stored late.
	// 0 with a model, whose chunk-0 update needs the bit offset first.
	// (AUTO: two images, so that four workgroups fit a CU with 32-bit images)
	constexpr uint32_t NIMG = AUTOK ? 2u : seg_images(W, MODEL);
	// With a model the update of chunk 0 needs the bit offset only to find the
	// samples the reference's loop never reached (fail_bit); FULL model
	// launches are host-checked to have no fail bit, so their look-back
	// overlaps the packing like the others
	constexpr uint32_t LBC = ((MODEL && !FULL) || CH < 2) ? 0u : NIMG - 1u;
	constexpr uint32_t RW = EPT * W / 16u; // uint4 per lane per chunk
	constexpr uint32_t MRW = EPT / 8u;      // uint4 of 16-bit model values per lane per chunk
	constexpr bool EXT_HDR = !(PRE == PRE_NONE && ENC == ENC_RAW);
	// STREAM (payload-only, cmp_gpu_encode_stream): one frame without header
	// or checksum, its bit stream starting at bit 0 of dst
	constexpr uint32_t HDR_BITS = STREAM ? 0u : EXT_HDR ? 176u : 128u;
	// NIMG chunk images in dynamic LDS, a.img_words each (sized per launch from
	// the longest codeword the pass can emit), each after a 4-word guard
	extern __shared__ __attribute__((aligned(16))) uint32_t L_dyn[];
	const uint32_t IMGW = a.img_words + 4u; // words per image incl. guard (multiple of 4)
	__shared__ uint32_t s_wsum[CH][EWG / 64];
	__shared__ uint32_t s_misc[8];
	// Rice/ZERO code table (fast path): entry q' = min(q, 17) holds
	// {T'[q'], len[q']} with codeword = m + T'[q'] (see rice_table)
	__shared__ __attribute__((aligned(16))) uint2 s_rice[20];

	const uint32_t tid = threadIdx.x, lane = tid & 63u;
	if (DBG(16384u)) // ablation: empty kernel
		return;
	const uint32_t wid = __builtin_amdgcn_readfirstlane(tid >> 6); // wave-uniform

	// ---- segment id: dispatch order (or an atomic ticket, debug switch) ----
	uint32_t seg = blockIdx.x;
	if (DBG(4u)) {
		if (tid == 0)
			s_misc[0] = atomicAdd(a.ticket, 1u) - a.ticket_base;
		__syncthreads();
		seg = __builtin_amdgcn_readfirstlane(s_misc[0]);
	}
	// Frame-interleaved dispatch: consecutive blocks take the same segment
	// index of consecutive frames.  A frame's segments are still dispatched in
	// order (a look-back only waits on earlier blocks) while the segments in
	// flight spread over all frames, keeping each look-back chain short.
	// AUTO: frame-major instead, so that a frame's segments (which all wait
	// for each other's Rice candidates) are dispatched together, and on one
	// XCD: blocks b, b + 8, b + 16, ... share an XCD (MI355X_MICROARCH.md,
	// dispatch), so frame 8 j + x takes blocks x + 8 (j spf + s), s < spf.
	// The grid is padded to whole groups of 8 frames.
	const uint32_t nfr = a.num_segs / a.segs_per_frame;
	uint32_t sif, lf;
	if (AUTOK) {
		const uint32_t p = seg >> 3;
		sif = p % a.segs_per_frame;
		lf = 8u * (p / a.segs_per_frame) + (seg & 7u);
		if (lf >= nfr)
			return; // padding block (uniform: the whole workgroup)
	} else {
		sif = seg / nfr;
		lf = seg - sif * nfr;
	}
	const uint32_t gseg = lf * a.segs_per_frame + sif; // granule slot: frame-major
	const uint32_t frame =
		__builtin_amdgcn_readfirstlane(a.frame_list ? a.frame_list[lf] : a.frame_add + lf * a.frame_mul);
	// a hole in a device-planned launch list (batch fallback path: the
	// context takes the other pass this step, or none): the whole frame is
	// skipped, and no segment of another frame waits on it
	if (frame == AIRS_NO_FRAME)
		return;
	const bool is_first = sif == 0u;
	const bool is_last = sif + 1u == a.segs_per_frame;
	const uint32_t n = a.n;
	dbg_stamp(a, gseg, 0);

	const uint8_t *fsrc = a.src + (uint64_t)frame * a.src_stride;
	// PRE_IWT: the residuals are the frame's IWT coefficients, computed into
	// the work buffer by iwt_frame_kernel (reference preprocess.c:321-353);
	// the samples themselves are only needed to store the model (MODEL == 1)
	constexpr bool LOADM = MODEL == 2 || PRE == PRE_IWT;
	constexpr bool NEEDX = !(PRE == PRE_IWT && MODEL == 0);
	uint8_t *fmodel = nullptr;
	if (MODEL || PRE == PRE_IWT)
		fmodel = a.model_ptrs ? reinterpret_cast<uint8_t *>(a.model_ptrs[lf])
				      : a.model + (uint64_t)(frame / a.model_div) * a.model_stride;
	// FULL launches (host-checked): every segment is whole and every frame and
	// model base is 16-byte aligned, so no per-lane bounds or alignment tests
	const bool src_al = FULL || ((uintptr_t)fsrc & 15u) == 0;
	const bool mod_al = (MODEL || PRE == PRE_IWT) ? (FULL || ((uintptr_t)fmodel & 15u) == 0) : true;

	// ---- phase 0: issue every load of the segment -----------------------
	uint32_t firstc[CH];
	uint4 raw[CH][RW];
	uint4 mraw[CH][MRW];
	uint32_t prevld[CH];
#pragma unroll
	for (uint32_t c = 0; c < CH; c++) {
		firstc[c] = sif * SEGN + c * AIRS_SEG + tid * EPT;
		const bool full = FULL || firstc[c] + EPT <= n;
		if (NEEDX && full && src_al) {
			const uint4 *p = reinterpret_cast<const uint4 *>(fsrc + (size_t)firstc[c] * W);
			if (DBG(512u)) { // ablation: no HBM reads (synthetic in-register data)
#pragma unroll
				for (uint32_t q = 0; q < RW; q++)
					raw[c][q] = make_uint4(0x40004000u + tid * 3u + q, 0x40104008u + c, 0x40204010u ^ tid,
							       0x40304018u + q * 7u);
			} else {
#pragma unroll
				for (uint32_t q = 0; q < RW; q++)
					raw[c][q] = p[q];
			}
		}
		if (LOADM && full && mod_al) {
			const uint4 *p = reinterpret_cast<const uint4 *>(fmodel + (size_t)firstc[c] * 2u);
#pragma unroll
			for (uint32_t q = 0; q < MRW; q++)
				mraw[c][q] = p[q];
		}
		prevld[c] = 0u;
		if (PRE == PRE_DIFF && lane == 0u && firstc[c] != 0u && firstc[c] <= n && !(DBG(512u)))
			prevld[c] = W == 2 ? (uint32_t)reinterpret_cast<const uint16_t *>(fsrc)[firstc[c] - 1u]
					   : reinterpret_cast<const uint32_t *>(fsrc)[firstc[c] - 1u] & 0xFFFFu;
	}

	// zero both LDS chunk images while the loads are in flight
	{
		uint4 *L4 = reinterpret_cast<uint4 *>(L_dyn);
		const uint32_t nz = AUTOK && NIMG * IMGW < AUTO_BINS * 64u ? AUTO_BINS * 64u : NIMG * IMGW;
		for (uint32_t i = tid; i < ((DBG(4096u)) ? 0u : nz / 4u); i += EWG)
			L4[i] = make_uint4(0u, 0u, 0u, 0u);
	}

	// (AUTO: set once the frame's k is known, after the residuals)
	uint32_t gpar = AUTOK ? 1u : __builtin_amdgcn_readfirstlane(a.frame_g ? a.frame_g[frame] : a.g);
	Coder cd = make_coder<ENC>(ENC == ENC_RAW ? 1u : gpar, a.outlier_param);

	// ---- phase 1: residuals, mapped values, code lengths ------------------
	// Samples are handled as packed 16-bit pairs: DIFF is one v_pk_sub_u16
	// against the pair shifted by one sample (v_alignbit), ZigZag three
	// packed ops, and for Rice/ZERO with k <= 11 the code lengths are summed
	// with packed ops too (length = k + 1 + min((m + 1) >> k, 16)).
	bool fastk = ENC == ENC_ZERO && RICE && cd.k <= 11u;
	if (!AUTOK && fastk && tid < 18u)
		s_rice[tid] = rice_table_entry(tid, cd.k);
	uint32_t mp[CH][EPT / 2]; // mapped values, two 16-bit per register
	// Rice/ZERO fast path (AIRS_KEEP_Q): the code-table byte offsets
	// 8 min(q, 17) of every pair, computed once in phase 1 next to the lengths
#ifndef AIRS_KEEP_Q
#define AIRS_KEEP_Q 1
#endif
	uint32_t mq[AIRS_KEEP_Q ? CH : 1][EPT / 2];
	uint32_t nmp[MODEL ? CH : 1][EPT / 2]; // new model values (MODEL)
	uint32_t T[CH], nv[CH];
	// code lengths of chunk c (T[c]) and, on the Rice/ZERO table path, the
	// table offsets of its samples (mq[c]), from the mapped values mp[c]
	auto lengths = [&](uint32_t c) {
		uint32_t t = 0u;
		if (DBG(64u)) {
			t = EPT * (cd.k + 1u) + (mp[c][0] & 7u);
		} else if (fastk && nv[c] == EPT) {
			u16x2 acc = (u16x2)(0);
#pragma unroll
			for (uint32_t j = 0; j < EPT / 2; j++) {
				const u16x2 v = __builtin_elementwise_add_sat(pk(mp[c][j]), (u16x2)(1));
				const u16x2 q = v >> (u16x2)((unsigned short)cd.k);
				acc += __builtin_elementwise_min(q, (u16x2)(16));
				if (AIRS_KEEP_Q)
					mq[AIRS_KEEP_Q ? c : 0][j] = unpk(__builtin_elementwise_min(q, (u16x2)(17)) << (u16x2)(3));
			}
			t = EPT * (cd.k + 1u) + (unpk(acc) & 0xFFFFu) + (unpk(acc) >> 16);
		} else {
#pragma unroll
			for (uint32_t j = 0; j < EPT; j++)
				t += j < nv[c] ? len_from_m<ENC, RICE>(half16(mp[c][j >> 1], j & 1u), cd) : 0u;
		}
		T[c] = t;
	};
#pragma unroll
	for (uint32_t c = 0; c < CH; c++) {
		const uint32_t first = firstc[c];
		nv[c] = FULL ? (uint32_t)EPT : first >= n ? 0u : min(n - first, (uint32_t)EPT);
		uint32_t w[EPT / 2]; // sample pairs (x[2j] | x[2j+1] << 16)
		if (!NEEDX) {
#pragma unroll
			for (uint32_t j = 0; j < EPT / 2; j++)
				w[j] = 0u;
		} else if (nv[c] == EPT && src_al) {
			if (W == 2) {
#pragma unroll
				for (uint32_t q = 0; q < RW; q++) {
					w[4 * q] = raw[c][q].x;
					w[4 * q + 1] = raw[c][q].y;
					w[4 * q + 2] = raw[c][q].z;
					w[4 * q + 3] = raw[c][q].w;
				}
			} else {
#pragma unroll
				for (uint32_t q = 0; q < RW; q++) {
					w[2 * q] = __builtin_amdgcn_perm(raw[c][q].y, raw[c][q].x, 0x05040100u);
					w[2 * q + 1] = __builtin_amdgcn_perm(raw[c][q].w, raw[c][q].z, 0x05040100u);
				}
			}
		} else {
#pragma unroll
			for (uint32_t j = 0; j < EPT / 2; j++) {
				uint32_t x2[2];
#pragma unroll
				for (uint32_t h = 0; h < 2; h++) {
					const uint32_t i = first + 2 * j + h;
					x2[h] = i < n ? (W == 2 ? (uint32_t)reinterpret_cast<const uint16_t *>(fsrc)[i]
								: reinterpret_cast<const uint32_t *>(fsrc)[i] & 0xFFFFu)
						      : 0u;
				}
				w[j] = x2[0] | x2[1] << 16;
			}
		}
		uint32_t pm[EPT / 2]; // model pairs (MODEL == 2) or IWT coefficient pairs
		if (LOADM) {
			if (nv[c] == EPT && mod_al) {
#pragma unroll
				for (uint32_t q = 0; q < MRW; q++) {
					pm[4 * q] = mraw[c][q].x;
					pm[4 * q + 1] = mraw[c][q].y;
					pm[4 * q + 2] = mraw[c][q].z;
					pm[4 * q + 3] = mraw[c][q].w;
				}
			} else {
#pragma unroll
				for (uint32_t j = 0; j < EPT / 2; j++) {
					uint32_t x2[2];
#pragma unroll
					for (uint32_t h = 0; h < 2; h++) {
						const uint32_t i = first + 2 * j + h;
						x2[h] = i < n ? (uint32_t)reinterpret_cast<const uint16_t *>(fmodel)[i] : 0u;
					}
					pm[j] = x2[0] | x2[1] << 16;
				}
			}
		}
		uint32_t wprev = 0u; // pair whose high half is the sample before this lane's first
		if (PRE == PRE_DIFF) {
			wprev = __shfl_up(w[EPT / 2 - 1], 1, 64);
			if (lane == 0u)
				wprev = prevld[c] << 16;
		}
#pragma unroll
		for (uint32_t j = 0; j < EPT / 2; j++) {
			uint32_t u;
			if (PRE == PRE_DIFF)
				u = unpk(pk(w[j]) - pk(__builtin_amdgcn_alignbit(w[j], j ? w[j - 1] : wprev, 16)));
			else if (PRE == PRE_MODEL)
				u = unpk(pk(w[j]) - pk(pm[j]));
			else if (PRE == PRE_IWT)
				u = pm[j];
			else
				u = w[j];
			mp[c][j] = (DBG(8192u)) ? w[j] : (ENC == ENC_RAW ? u : zigzag_pk(u));
		}
		if (!AUTOK)
			lengths(c);
		if (MODEL) {
#pragma unroll
			for (uint32_t j = 0; j < EPT / 2; j++) {
				if (MODEL == 1) {
					nmp[MODEL ? c : 0][j] = w[j];
				} else {
					// cmp.c:132-142
					nmp[MODEL ? c : 0][j] = model_update_pk(w[j], pm[j], a.is_unsigned ? 0u : 0x80008000u,
										16 - (int32_t)a.model_rate);
				}
			}
		}
		// Make the packed mapped values opaque: otherwise the compiler keeps
		// phase 1's per-sample intermediates alive to CSE them with phase 2's
		// recomputation, which costs ~100 extra VGPRs and halves occupancy.
#pragma unroll
		for (uint32_t i = 0; i < EPT / 2; i++)
			asm volatile("" : "+v"(mp[c][i]));
		if (AIRS_KEEP_Q && !AUTOK) {
#pragma unroll
			for (uint32_t i = 0; i < EPT / 2; i++)
				asm volatile("" : "+v"(mq[AIRS_KEEP_Q ? c : 0][i]));
		}
	}

	uint32_t auto_P = 0u; // AUTO: the segment's frame bit offset (header included)
	if constexpr (AUTOK) {
		// ---- the frame's Rice k ---------------------------
		// 1. histogram: one 32-bit counter per (bin, lane of the wave), shared
		// by the four waves (atomic, no return), bank = lane: conflict-free.
		// It lives in the (zeroed) chunk images, which are not in use yet.
		__shared__ uint32_t s_hist[AUTO_BINS];
		__shared__ uint32_t s_kt[EWG / 64][16];
		uint32_t *const H = L_dyn;
		// this lane's counter of bin b is at byte hbase + 256 (b + 1016): the
		// bin's offset comes from the float bits with one (full-rate) shift
		// and one shift-add (32-bit LDS address arithmetic wraps)
		const uint32_t hbase = (uint32_t)(uintptr_t)H + 4u * lane - 1016u * 256u;
		__syncthreads(); // the images are zeroed
#pragma unroll
		for (uint32_t c = 0; c < CH; c++) {
#pragma unroll
			for (uint32_t jp = 0; jp < EPT / 2; jp++) {
				// an opaque copy of the pair: otherwise the compiler computes
				// all 64 bins ahead of the barrier above (~150 more VGPRs)
				uint32_t wv = mp[c][jp];
				asm volatile("" : "+v"(wv));
#pragma unroll
				for (uint32_t h = 0; h < 2; h++) {
					const uint32_t j = 2u * jp + h;
					if ((FULL || j < nv[c]) && !AIRS_AUTO_ABL(1)) {
						const uint32_t v = half16(wv, h) + 1u;
						// (as asm: the compiler turns the pair into shift, and, add)
						uint32_t ha;
						asm("v_lshrrev_b32 %0, 20, %1\n\tv_lshl_add_u32 %0, %0, 8, %2"
						    : "=&v"(ha)
						    : "v"(__float_as_uint((float)v)), "v"(hbase));
						lds_u32 *hp = reinterpret_cast<lds_u32 *>((uintptr_t)ha);
						__hip_atomic_fetch_add(hp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
					}
				}
			}
		}
		__syncthreads();
		dbg_stamp(a, gseg, 5);
		// 2. bin totals: threads 2r, 2r+1 sum the halves of row r < 128 with
		// eight 16-byte reads each, rotated by r (4-way bank sharing); wave 0
		// sums row 128 (v = 65536)
		{
			const uint32_t r = tid >> 1, h = tid & 1u;
			const uint4 *row = reinterpret_cast<const uint4 *>(H + r * 64u + h * 32u);
			uint32_t s = 0u;
#pragma unroll
			for (uint32_t hq = 0; hq < 8u; hq += 4u) {
				uint4 q4[4];
#pragma unroll
				for (uint32_t q = 0; q < 4u; q++)
					q4[q] = row[(hq + q + r) & 7u];
#pragma unroll
				for (uint32_t q = 0; q < 4u; q++)
					s += q4[q].x + q4[q].y + q4[q].z + q4[q].w;
				__builtin_amdgcn_sched_barrier(0);
			}
			s += __shfl_xor(s, 1, 64);
			if (h == 0u)
				s_hist[r] = s;
			static_assert(AUTO_BINS == EWG / 2u + 1u, "rows 0..127 by thread pairs, then row 128");
			if (wid == 0) {
				const uint32_t s128 = wave_sum(H[128u * 64u + lane]);
				if (lane == 0)
					s_hist[128] = s128;
			}
		}
		__syncthreads();
		// the images again as images: clear the histogram rows
		for (uint32_t i = tid; i < AUTO_BINS * 64u / 4u; i += EWG)
			reinterpret_cast<uint4 *>(H)[i] = make_uint4(0u, 0u, 0u, 0u);
		// 3. this segment's 16 candidate sums: thread (slice s, k) covers bins
		// s, s + 16, ...; the four slices of a wave meet through two shuffles
		{
			const uint32_t k = tid & 15u, sl = tid >> 4;
			uint32_t part = 0u;
#pragma unroll
			for (uint32_t i = 0; i < (AUTO_BINS + 15u) / 16u; i++) {
				const uint32_t b = sl + 16u * i;
				if (b < AUTO_BINS)
					part += s_hist[b] * auto_term(b, k);
			}
			part += __shfl_xor(part, 16, 64);
			part += __shfl_xor(part, 32, 64);
			if (lane < 16u)
				s_kt[wid][k] = part;
		}
		__syncthreads();
		if (wid == 0) {
			// 4. publish (lanes 0-15), then read the frame's 16 * spf granules
			if (lane < 16u) {
				const uint32_t sk = s_kt[0][lane] + s_kt[1][lane] + s_kt[2][lane] + s_kt[3][lane];
				gran_store(&a.ktot[(uint64_t)gseg * 16u + lane], ((uint64_t)a.epoch << 32) | sk);
			}
			const uint32_t first_seg = gseg - sif, ng = a.segs_per_frame * 16u;
			constexpr uint32_t NL = (AUTO_MAX_SPF + 3u) / 4u; // granule loads per lane
			uint64_t gk[NL];
#pragma unroll
			for (uint32_t i = 0; i < NL; i++) {
				const uint32_t gi = 64u * i + lane;
				gk[i] = gran_load(&a.ktot[(uint64_t)first_seg * 16u + (gi < ng ? gi : 0u)]);
			}
			uint32_t spins = 0u;
			for (; !AIRS_AUTO_ABL(2);) {
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
						gk[i] = gran_load(&a.ktot[(uint64_t)first_seg * 16u + gi]);
				}
			}
			// lane l holds segment 4i + l/16, candidate k = l % 16
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
			const uint32_t k = lane & 15u;
			// frame bits for k (< 2^28: spf <= 32 segments), ties to the smaller k
			uint32_t key = ((tot + n * (k + 1u)) << 4) | k;
#pragma unroll
			for (uint32_t d = 1; d < 16u; d <<= 1)
				key = min(key, (uint32_t)__shfl_xor(key, d, 64));
			const uint32_t ks = key & 15u;
			const uint32_t pre_k = __shfl(pre, ks, 64);
			if (lane == 0) {
				s_misc[4] = ks;
				// every segment before this one is whole
				s_misc[5] = HDR_BITS + pre_k + sif * SEGN * (ks + 1u);
			}
		}
		__syncthreads();
		dbg_stamp(a, gseg, 6);
		const uint32_t ks = __builtin_amdgcn_readfirstlane(s_misc[4]);
		auto_P = __builtin_amdgcn_readfirstlane(s_misc[5]);
		gpar = 1u << ks;
		cd = make_coder<ENC>(gpar, a.outlier_param);
		fastk = ks <= 11u;
		if (fastk && tid < 18u)
			s_rice[tid] = rice_table_entry(tid, ks);
#pragma unroll
		for (uint32_t c = 0; c < CH; c++) {
			lengths(c);
			if (AIRS_KEEP_Q) {
#pragma unroll
				for (uint32_t i = 0; i < EPT / 2; i++)
					asm volatile("" : "+v"(mq[AIRS_KEEP_Q ? c : 0][i]));
			}
		}
	}

	if (DBG(32768u)) { // ablation: stop after phase 1
		if (T[0] == 0x12345u && tid == 999u)
			a.status[0] = mp[0][0] + mp[CH - 1][1];
		return;
	}
	// ---- per-chunk block scans (DPP within waves, LDS across waves) -------
	uint32_t inc[CH];
#pragma unroll
	for (uint32_t c = 0; c < CH; c++) {
		inc[c] = wave_incl_scan(T[c]);
		if (lane == 63u)
			s_wsum[c][wid] = inc[c];
	}

	// ---- the segment's last 32 bits (wave 3 rebuilds its last chunk) ------
#ifndef AIRS_LB_WIN
#define AIRS_LB_WIN 1
#endif
	// look-back windows of 64 granules fetched per round.  A stream is one
	// frame with ~1024 segments in flight (not ~64); it used four windows
	// (256 segments back per round), but one window is 12 % faster on the
	// 64 Mi-sample stream (cold A/B on one box: 64.9 vs 73.5-74.5 us,
	// DESIGN.md 3.1.2): the extra windows only add loads to the round
#ifndef AIRS_STREAM_LB_WIN
#define AIRS_STREAM_LB_WIN 1
#endif
	constexpr int LB_WIN = STREAM ? AIRS_STREAM_LB_WIN : AIRS_LB_WIN;
	// Scalar look-back (experiment, AIRS_SLB=1): the first round reads the
	// 16 newest granules and the tail through the scalar cache path (glc:
	// no scalar-cache hit) when the look-back starts, instead of vector loads
	// issued a chunk earlier that queue behind the CU's cold sample loads.
	// A stale or unpublished granule only means another round (vector).
#ifndef AIRS_SLB
#define AIRS_SLB 1
#endif
#ifndef AIRS_SLB_N
#define AIRS_SLB_N 16
#endif
	constexpr bool SLB = AIRS_SLB && LBC >= 1 && !AUTOK;
	constexpr uint32_t SLB_N = AIRS_SLB_N; // 8, 16 or 32 granules
	uint64_t gv[LB_WIN];
#pragma unroll
	for (int w = 0; w < LB_WIN; w++)
		gv[w] = 0;
	__syncthreads(); // B1: wave totals visible
	uint32_t excl[CH], tot[CH], base[CH];
	uint32_t A = 0u;
#pragma unroll
	for (uint32_t c = 0; c < CH; c++) {
		uint32_t woff = 0u, tt = 0u;
#pragma unroll
		for (uint32_t w = 0; w < EWG / 64; w++) {
			const uint32_t v = s_wsum[c][w];
			woff += w < wid ? v : 0u;
			tt += v;
		}
		excl[c] = woff + inc[c] - T[c];
		tot[c] = __builtin_amdgcn_readfirstlane(tt); // LDS-loaded, but block-uniform
		base[c] = A;
		A += tt;
	}
	const uint32_t first_seg = gseg - sif;
	uint64_t tv0 = 0; // predecessor's tail granule, fetched early (lane 0 of wave 0)
	if (wid == 0) {
		if (lane == 0 && !AUTOK) {
			const uint64_t tag = ((uint64_t)a.epoch << 1) | (is_first ? 1u : 0u);
			gran_store(&a.agg[gseg], (tag << 32) | (is_first ? HDR_BITS + A : A));
		}
		dbg_stamp(a, gseg, 1);
		if (LBC == 0 && !is_first && !(DBG(2u)) && !AUTOK) {
			// the first round's windows, newest first: with ~64 segments of a
			// frame in flight the nearest inclusive prefix is often past 64
			lb_prefetch<LB_WIN>(a, gv, tv0, gseg, first_seg, lane);
		}
	}
	if (!is_last && wid == EWG / 64 - 1 && !(DBG(8u))) {
		// the last lanes' streams (>= EPT bits each) combined: lane 63 gets
		// the chunk's last 32 bits
		uint64_t acc = 0u;
		if (fastk && nv[CH - 1] == EPT) {
			const char *tab = reinterpret_cast<const char *>(s_rice);
			auto pair = [&](uint32_t j) {
				u16x2 qa;
				if (AIRS_KEEP_Q) {
					qa = pk(mq[AIRS_KEEP_Q ? CH - 1 : 0][j]);
				} else {
					const u16x2 v = __builtin_elementwise_add_sat(pk(mp[CH - 1][j]), (u16x2)(1));
					qa = __builtin_elementwise_min(v >> (u16x2)((unsigned short)cd.k), (u16x2)(17)) << (u16x2)(3);
				}
#pragma unroll
				for (uint32_t h = 0; h < 2; h++) {
					const uint2 e = *reinterpret_cast<const uint2 *>(tab + half16(unpk(qa), h));
					acc = (acc << e.y) | (half16(mp[CH - 1][j], h) + e.x);
				}
			};
			// every sample takes >= k + 1 bits, so for k >= 3 the lane's last
			// 32 bits lie in its last 8 samples: the first pairs are skipped
			if (EPT >= 16 && cd.k >= 3u) {
#pragma unroll
				for (uint32_t j = EPT / 4; j < EPT / 2; j++)
					pair(j);
			} else {
#pragma unroll
				for (uint32_t j = 0; j < EPT / 2; j++)
					pair(j);
			}
		} else {
#pragma unroll
			for (uint32_t j = 0; j < EPT; j++) {
				const uint32_t m = (mp[CH - 1][j >> 1] >> (16u * (j & 1u))) & 0xFFFFu;
				uint32_t c1, l1, c2, l2;
				code_from_m<ENC, RICE>(m, cd, c1, l1, c2, l2);
				acc = (acc << l1) | c1;
				if (NPIECE == 2)
					acc = (acc << l2) | c2;
			}
		}
		// (v, t) = the last min(T, 32) stream bits of a lane run; combining an
		// earlier run a with a later b is associative: two scan steps cover
		// four lanes, >= 32 bits for EPT >= 8
		uint32_t v = (uint32_t)acc, tb = min(T[CH - 1], 32u);
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

	uint32_t last_ne = 0u; // last non-empty chunk
#pragma unroll
	for (uint32_t c = 0; c < CH; c++)
		last_ne = tot[c] ? c : last_ne;

	uint8_t *fdst = a.dst + (uint64_t)frame * a.dst_stride;
	const uint32_t cap = a.cap;
	const __amdgpu_buffer_rsrc_t dst_rsrc = __builtin_amdgcn_make_buffer_rsrc(fdst, 0, (int)(cap & ~3u), 0x00020000);
	uint32_t P = 0u;
	uint32_t pred_c = 0u; // (lane 0 of wave 0) bits preceding chunk c in its first dword
	const uint32_t tot_first = tot[0];

	// Store one chunk image: funnel-shift it to its frame bit offset.  Complete
	// words go out through a buffer descriptor whose range is the frame's
	// capacity rounded down to whole words, so the hardware range check drops
	// exactly the words that would not fit.
	auto store_chunk = [&](const uint32_t *Lx, uint32_t basex, uint32_t totx, uint32_t predx, bool finalx) {
		if (!totx)
			return;
		const uint32_t Pc = P + basex;
		const uint32_t r = Pc & 31u, g0 = Pc >> 5;
		const uint32_t endbit = Pc + totx;
		const uint32_t J = ((endbit - 1u) >> 5) - g0; // last word touched
		const uint32_t nfull = (endbit & 31u) == 0u ? J + 1u : J;
		// four words per thread: one 16-byte LDS read + its left neighbour, one
		// 16-byte buffer store (the image is 16-byte aligned, j a multiple of 4)
		const lds_u32 *Ll = reinterpret_cast<const lds_u32 *>((uintptr_t)Lx);
		const uint32_t nquad = (DBG(2048u)) ? 0u : (nfull >> 2);
		for (uint32_t p = tid; p < nquad; p += EWG) {
			const uint32_t j = 4u * p;
			const u32x4 w = *reinterpret_cast<const __attribute__((address_space(3))) u32x4 *>(Ll + j);
			const uint32_t hi = j ? Ll[j - 1u] : predx;
			u32x4 o;
			o.x = bswap32(__builtin_amdgcn_alignbit(hi, w.x, r));
			o.y = bswap32(__builtin_amdgcn_alignbit(w.x, w.y, r));
			o.z = bswap32(__builtin_amdgcn_alignbit(w.y, w.z, r));
			o.w = bswap32(__builtin_amdgcn_alignbit(w.z, w.w, r));
			if (!(DBG(1024u))) // ablation: no HBM writes
				__builtin_amdgcn_raw_buffer_store_b128(o, dst_rsrc, (int)(4u * (g0 + j)), 0, 0);
		}
		// the last nfull % 4 words: one each for the threads next in turn
		// (thread 0 when one of them is word 0, the only word that needs
		// predx, which lives in lane 0 of wave 0)
		const uint32_t rr = (tid - nquad) & (EWG - 1u);
		if (rr < (nfull & 3u) && !(DBG(2048u))) {
			const uint32_t j = 4u * nquad + rr;
			const uint32_t hi = j ? Ll[j - 1u] : predx;
			const uint32_t v = __builtin_amdgcn_alignbit(hi, Ll[j], r);
			if (!(DBG(1024u)))
				__builtin_amdgcn_raw_buffer_store_b32(bswap32(v), dst_rsrc, (int)(4u * (g0 + j)), 0, 0);
		}
		if (finalx && nfull == J && tid == 0) {
			// zero-padded final bytes of the payload (reference bitstream_flush)
			const uint32_t hi = J ? Lx[J - 1u] : predx;
			const uint32_t v = __builtin_amdgcn_alignbit(hi, Lx[J], r);
			const uint32_t gw = g0 + J;
			const uint32_t nbytes = ((endbit & 31u) + 7u) >> 3;
			for (uint32_t b = 0; b < nbytes; b++)
				if (4u * gw + b < cap)
					fdst[4u * gw + b] = (uint8_t)(v >> (24u - 8u * b));
		}
	};

	// ---- phase 2: chunk by chunk: codewords -> LDS image -> HBM -----------
	// Waves past phase 1 issue ahead of waves of newer segments on the same
	// SIMD (still in phase 1): the older segment holds LDS and its frame's
	// look-back chain, so finishing it first shortens residency (measured:
	// 1-3 % on cfg2 and the cfg4 shard).
#ifndef AIRS_PRIO_P2
#define AIRS_PRIO_P2 1
#endif
	if (AIRS_PRIO_P2)
		__builtin_amdgcn_s_setprio(AIRS_PRIO_P2);
	// rolled loop (keeps register pressure flat): the current chunk's state is
	// always index 0 of mp/nmp/nv/excl/tot/base/firstc, rotated at the end
	uint32_t tot_m3 = 0u; // totals of chunks c-3, c-2 (an image is recycled now), c-1
	uint32_t tot_m2 = 0u;
	uint32_t tot_m1 = 0u;
	uint32_t pred_1 = 0u; // (tid 0) last 32 bits of chunk 0, kept for chunk 1's late store
	uint32_t pred_2 = 0u; // (tid 0) last 32 bits of chunk 1 (four images: chunk 2 is stored late too)
#ifndef AIRS_CHUNK_UNROLL
#define AIRS_CHUNK_UNROLL 4
#endif
#pragma unroll AIRS_CHUNK_UNROLL
	for (uint32_t c = 0; c < CH; c++) {
		uint32_t *Lc = L_dyn + (c % NIMG) * IMGW + 4u;
		if (LBC >= 1 && c == LBC + 1u && c >= NIMG)
			__syncthreads(); // chunk 0's image was stored (late) after the last barrier
		if (c >= NIMG) {
			// image c%NIMG was last read by chunk c-NIMG's stores (before the
			// barrier that ended chunk c-1's packing): clear what it used
			const uint32_t nw = (max(NIMG == 2 ? tot_m2 : tot_m3, tot[0]) + 31u) >> 5;
			for (uint32_t i = tid; i <= ((DBG(4096u)) ? 0u : nw); i += EWG)
				Lc[i] = 0u;
			__syncthreads();
		}
#ifndef AIRS_LBP
#define AIRS_LBP LBC
#endif
		if (LBC >= 1 && c == (AIRS_LBP) && wid == 0 && !is_first && !(DBG(2u))) {
			if (AUTOK) // only the predecessor's tail: the offset is known
				tv0 = gran_load(&a.tail[gseg - 1u]);
			else if (!SLB || sif < SLB_N)
				lb_prefetch<LB_WIN>(a, gv, tv0, gseg, first_seg, lane);
		}
		uint32_t ln[NPIECE][EPT]; // piece lengths (kept for the MODEL fail_bit check)
		{
			Packer pk1;
			pk1.init(Lc, excl[0]);
			if (DBG(32u)) {
			} else if (fastk && nv[0] == EPT) {
				// table-driven: byte offsets 8*min(q, 17) of both samples of a
				// pair come from three packed ops; codeword = m + T'[q']
				// (all 16 lookups are issued before the first put: the compiler
				// does not move LDS reads across the packer's ds_or atomics)
				const char *tab = reinterpret_cast<const char *>(s_rice);
#pragma unroll
				for (uint32_t hb = 0; hb < 2; hb++) { // two batches of 8 lookups
					uint2 te[EPT / 2];
#pragma unroll
					for (uint32_t jj = 0; jj < EPT / 4; jj++) {
						const uint32_t j = hb * (EPT / 4) + jj;
						u16x2 qa;
						if (AIRS_KEEP_Q) {
							qa = pk(mq[0][j]);
						} else {
							const u16x2 v = __builtin_elementwise_add_sat(pk(mp[0][j]), (u16x2)(1));
							qa = __builtin_elementwise_min(v >> (u16x2)((unsigned short)cd.k), (u16x2)(17))
							     << (u16x2)(3);
						}
#pragma unroll
						for (uint32_t h = 0; h < 2; h++)
							te[2 * jj + h] = *reinterpret_cast<const uint2 *>(tab + half16(unpk(qa), h));
					}
					// both codewords of a pair go in one put when they fit in 32
					// bits (almost always).  The test is made once per batch for
					// the whole wave (one ballot, a uniform branch): if any lane
					// has a longer pair, the whole batch takes two puts per pair.
					uint32_t mxl = 0u;
#pragma unroll
					for (uint32_t i = 0; i < EPT / 2; i += 2)
						mxl = max(mxl, te[i].y + te[i + 1].y);
					if (__ballot(mxl > 32u) == 0ull) {
#pragma unroll
						for (uint32_t i = 0; i < EPT / 2; i += 2) {
							const uint32_t j = hb * (EPT / 2) + i;
							const uint32_t cwa = (mp[0][j >> 1] & 0xFFFFu) + te[i].x;
							const uint32_t cwb = (mp[0][j >> 1] >> 16) + te[i + 1].x;
							pk1.put((cwa << te[i + 1].y) | cwb, te[i].y + te[i + 1].y);
						}
					} else {
#pragma unroll
						for (uint32_t i = 0; i < EPT / 2; i += 2) {
							const uint32_t j = hb * (EPT / 2) + i;
							pk1.put((mp[0][j >> 1] & 0xFFFFu) + te[i].x, te[i].y);
							pk1.put((mp[0][j >> 1] >> 16) + te[i + 1].x, te[i + 1].y);
						}
					}
#pragma unroll
					for (uint32_t i = 0; i < EPT / 2; i += 2) {
						const uint32_t j = hb * (EPT / 2) + i;
						ln[0][j] = te[i].y;
						ln[0][j + 1] = te[i + 1].y;
						if (NPIECE == 2) {
							ln[NPIECE - 1][j] = 0u;
							ln[NPIECE - 1][j + 1] = 0u;
						}
					}
				}
			} else {
#pragma unroll
				for (uint32_t j = 0; j < EPT; j++) {
					const uint32_t m = half16(mp[0][j >> 1], j & 1u);
					uint32_t c1, l1, c2, l2;
					code_from_m<ENC, RICE>(m, cd, c1, l1, c2, l2);
					const bool ok = j < nv[0];
					l1 = ok ? l1 : 0u;
					pk1.put(ok ? c1 : 0u, l1);
					ln[0][j] = l1;
					if (NPIECE == 2) {
						l2 = ok ? l2 : 0u;
						pk1.put(ok ? c2 : 0u, l2);
						ln[NPIECE - 1][j] = l2;
					}
				}
			}
			pk1.flush();
		}
		__syncthreads();
		uint32_t pred_next = 0u; // last 32 bits of this chunk, for chunk c+1 (tid 0)
		if (c + 1u < CH && tid == 0 && tot[0] >= 32u) {
			const uint32_t s0 = tot[0] - 32u, q = s0 >> 5, sh = s0 & 31u;
			pred_next = sh ? (Lc[q] << sh) | (Lc[q + 1] >> (32u - sh)) : Lc[q];
		}

		if (c == LBC) {
			// ---- decoupled look-back (wave 0), overlapped with the packing ----
			if (wid == 0) {
#ifdef AIRS_PRIO_LB // experiment: issue priority of the look-back wave
				__builtin_amdgcn_s_setprio(AIRS_PRIO_LB);
#endif
				dbg_stamp(a, gseg, 3);
				uint32_t Pw = HDR_BITS;
				if (AUTOK) {
					Pw = auto_P; // from the Rice candidates of the frame
				} else if (DBG(2u)) {
					Pw = HDR_BITS + sif * 37u; // ablation: no look-back (output garbage)
				} else if (!is_first) {
					// round 0 uses the granules fetched before packing; every
					// round covers LB_WIN windows of 64, newest first
					const bool slb = SLB && sif >= SLB_N;
					if (slb) {
						typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
						// (the addresses in SGPRs: uniform, but not known to be)
						auto sptr = [](const uint64_t *p) {
							const uint64_t v = (uint64_t)(uintptr_t)p;
							const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)v);
							const uint32_t h = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
							return (const uint64_t *)(uintptr_t)(((uint64_t)h << 32) | l);
						};
						const uint64_t *gp = sptr(&a.agg[gseg - SLB_N]);
						const uint64_t *tp = sptr(&a.tail[gseg - 1u]);
						// q[b] = granules gseg - SLB_N + 8 b .. + 7; the loads and their
						// wait in one statement (lgkmcnt also counts LDS operations)
						u32x16 q[SLB_N / 8u];
						uint64_t tq;
						if constexpr (SLB_N == 32u)
							asm volatile("s_load_dwordx16 %0, %5, 0x0 glc\n\t"
								     "s_load_dwordx16 %1, %5, 0x40 glc\n\t"
								     "s_load_dwordx16 %2, %5, 0x80 glc\n\t"
								     "s_load_dwordx16 %3, %5, 0xc0 glc\n\t"
								     "s_load_dwordx2 %4, %6, 0x0 glc\n\t"
								     "s_waitcnt lgkmcnt(0)"
								     : "=&s"(q[0]), "=&s"(q[1]), "=&s"(q[2]), "=&s"(q[3]), "=&s"(tq)
								     : "s"(gp), "s"(tp)
								     : "memory");
						else if constexpr (SLB_N == 8u)
							asm volatile("s_load_dwordx16 %0, %2, 0x0 glc\n\t"
								     "s_load_dwordx2 %1, %3, 0x0 glc\n\t"
								     "s_waitcnt lgkmcnt(0)"
								     : "=&s"(q[0]), "=&s"(tq)
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
						// granule gseg - SLB_N + i -> lane SLB_N - 1 - i; lanes >= SLB_N read
						// as unpublished (tag 0): they send the round to the vector path
						// unless an inclusive granule comes first
						uint32_t vl = 0u, vh = 0u;
#pragma unroll
						for (uint32_t i = 0; i < SLB_N; i++) {
							vl = lane == SLB_N - 1u - i ? q[i >> 3][2u * (i & 7u)] : vl;
							vh = lane == SLB_N - 1u - i ? q[i >> 3][2u * (i & 7u) + 1u] : vh;
						}
						gv[0] = ((uint64_t)vh << 32) | vl;
						tv0 = tq;
					}
					uint32_t sum = 0u, spins = 0u, lb_rounds = 0u;
					int64_t j = (int64_t)gseg - 1;
					int nwin = slb ? 1 : LB_WIN; // the scalar round fills one window
					bool done = false;
					while (!done) {
						lb_rounds++;
						bool retry = false;
#pragma unroll
						for (int w = 0; w < LB_WIN; w++) {
							if (w >= nwin || done || retry)
								break;
							const int64_t idx = j - 64 * w - (int64_t)lane;
							const bool inr = idx >= (int64_t)first_seg;
							const uint32_t tag = (uint32_t)(gv[w] >> 32);
							const bool valid = inr && (tag >> 1) == a.epoch;
							const bool incl = valid && (tag & 1u);
							const uint64_t incl_m = __ballot(incl);
							const uint64_t bad_m = __ballot(inr && !valid);
							const uint32_t fi =
								incl_m ? (uint32_t)__ffsll((unsigned long long)incl_m) - 1u : 64u;
							const uint64_t need = fi >= 63u ? ~0ull : ((2ull << fi) - 1ull);
							if (bad_m & need) {
								// a needed predecessor has not published: re-poll from here
								j -= 64 * w;
								retry = true;
								break;
							}
							sum += wave_sum((inr && lane <= fi) ? (uint32_t)gv[w] : 0u);
							if (incl_m)
								done = true;
						}
						if (done)
							break;
						if (retry) {
							if (++spins > AIRS_SPIN_LIMIT) {
								// never expected: a predecessor did not publish.  Give up
								// (output is garbage, the host reports the fault counter)
								if (lane == 0)
									atomicAdd(a.ticket + AIRS_FAULT_WORD, 1u);
								break;
							}
							__builtin_amdgcn_s_sleep(1);
						} else {
							j -= 64 * nwin;
						}
						nwin = LB_WIN;
#pragma unroll
						for (int w = 0; w < LB_WIN; w++) {
							const int64_t idx = j - 64 * w - (int64_t)lane;
							gv[w] = idx >= (int64_t)first_seg ? gran_load(&a.agg[idx]) : 0ull;
						}
					}
					Pw = sum;
					if (lane == 0)
						gran_store(&a.agg[gseg], ((((uint64_t)a.epoch << 1) | 1u) << 32) | (Pw + A));
					if ((DBG(65536u)) && a.dbgts && lane == 0)
						a.dbgts[8u * gseg + 5u] = ((uint64_t)spins << 32) | lb_rounds;
					if ((DBG(256u)) && lane == 0) { // look-back statistics (debug)
						atomicAdd(a.ticket + 20, 1u);
						atomicAdd(a.ticket + 21, lb_rounds);
						atomicAdd(a.ticket + 22, spins);
					}
				}
				if (lane == 0) {
					uint32_t pred = 0u;
					if (is_first || (DBG(2u))) {
						// header bytes 20-21 (low half of the outlier field) share
						// the first payload dword of a 22-byte header
						pred = (EXT_HDR && ENC != ENC_RAW && !STREAM) ? (cd.outlier & 0xFFFFu) : 0u;
					} else {
						uint64_t tv = tv0;
						uint32_t spins = 0;
						for (; (uint32_t)(tv >> 32) != a.epoch; spins++) {
							if (spins > AIRS_SPIN_LIMIT) {
								atomicAdd(a.ticket + AIRS_FAULT_WORD, 1u);
								break;
							}
							__builtin_amdgcn_s_sleep(1);
							tv = gran_load(&a.tail[gseg - 1u]);
							if (DBG(256u))
								atomicAdd(a.ticket + 23, 1u);
						}
						if ((DBG(65536u)) && a.dbgts && !AUTOK)
							a.dbgts[8u * gseg + 6u] = spins;
						pred = (uint32_t)tv;
					}
					s_misc[1] = Pw;
					s_misc[2] = pred;
				}
				dbg_stamp(a, gseg, 2);
#ifdef AIRS_PRIO_LB
				__builtin_amdgcn_s_setprio(AIRS_PRIO_P2);
#endif
			}
			__syncthreads();
			P = __builtin_amdgcn_readfirstlane(s_misc[1]);
			const uint32_t seg_pred = __builtin_amdgcn_readfirstlane(s_misc[2]);
			if (LBC == 0)
				pred_c = seg_pred;
			else if (tot_first) // chunk 0 waited for the look-back: store it now
				store_chunk(L_dyn + 4u, 0u, tot_first, seg_pred, is_last && last_ne == 0u);
			if (LBC == 2) // so did chunk 1
				store_chunk(L_dyn + IMGW + 4u, tot_first, tot_m1, pred_1, is_last && last_ne == 1u);
			if (LBC == 3) { // and, with four images, chunks 1 and 2
				store_chunk(L_dyn + IMGW + 4u, tot_first, tot_m2, pred_1, is_last && last_ne == 1u);
				store_chunk(L_dyn + 2u * IMGW + 4u, tot_first + tot_m2, tot_m1, pred_2,
					    is_last && last_ne == 2u);
			}
		}

		if (c >= LBC)
			store_chunk(Lc, base[0], tot[0], pred_c, is_last && c == last_ne);

		// ---- model update of chunk c (cmp.c:304-311), old model kept for the
		// samples the reference's loop never reached (see fail_bit) ----------
		if (MODEL && nv[0]) {
			uint64_t bpos = (uint64_t)P + base[0] + excl[0];
			bool all_ok = true;
			uint32_t okmask = 0u;
#pragma unroll
			for (uint32_t j = 0; j < EPT; j++) {
#pragma unroll
				for (uint32_t p = 0; p < NPIECE; p++)
					bpos += ln[p][j];
				const bool ok = j < nv[0] && bpos <= a.fail_bit;
				okmask |= ok ? (1u << j) : 0u;
				all_ok &= ok;
			}
			uint16_t *mpp = reinterpret_cast<uint16_t *>(fmodel) + firstc[0];
			if (all_ok && mod_al) {
				const uint32_t *q = nmp[0];
#pragma unroll
				for (uint32_t r = 0; r < MRW; r++)
					reinterpret_cast<uint4 *>(mpp)[r] = make_uint4(q[4 * r], q[4 * r + 1], q[4 * r + 2], q[4 * r + 3]);
			} else {
#pragma unroll
				for (uint32_t j = 0; j < EPT; j++)
					if (okmask & (1u << j))
						mpp[j] = (uint16_t)(nmp[0][j >> 1] >> (16u * (j & 1u)));
			}
		}
		if (c == 0)
			pred_1 = pred_next;
		if (c == 1)
			pred_2 = pred_next;
		pred_c = pred_next;
		// rotate the per-chunk state
		tot_m3 = tot_m2;
		tot_m2 = tot_m1;
		tot_m1 = tot[0];
#pragma unroll
		for (uint32_t k = 0; k + 1 < CH; k++) {
#pragma unroll
			for (uint32_t i = 0; i < EPT / 2; i++) {
				mp[k][i] = mp[k + 1][i];
				if (AIRS_KEEP_Q)
					mq[AIRS_KEEP_Q ? k : 0][i] = mq[AIRS_KEEP_Q ? k + 1 : 0][i];
				if (MODEL)
					nmp[k][i] = nmp[k + 1][i];
			}
			nv[k] = nv[k + 1];
			excl[k] = excl[k + 1];
			tot[k] = tot[k + 1];
			base[k] = base[k + 1];
			firstc[k] = firstc[k + 1];
		}
	}

	dbg_stamp(a, gseg, 4);
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
		header_words(h, size, 2u * n, id, a.seqs ? a.seqs[frame] : a.seq, PRE, a.checksum ? 1u : 0u, ENC,
			     PRE == PRE_MODEL ? a.model_rate : 0u, ENC == ENC_RAW ? 0u : gpar,
			     ENC == ENC_RAW ? 0u : cd.outlier);
		const uint32_t hwords = EXT_HDR ? 5u : 4u;
		if (((uintptr_t)fdst & 7u) == 0u && cap >= 4u * hwords) {
			// three stores instead of five (8-byte aligned frame): the partial
			// line shared with the frame's first segment; an ablation without
			// the header measured 1-2 us faster on cfg3/cfg4, this form the same
			// 
			*reinterpret_cast<uint2 *>(fdst) = make_uint2(bswap32(h[0]), bswap32(h[1]));
			*reinterpret_cast<uint2 *>(fdst + 8) = make_uint2(bswap32(h[2]), bswap32(h[3]));
			if (hwords == 5u)
				*reinterpret_cast<uint32_t *>(fdst + 16) = bswap32(h[4]);
		} else {
#pragma unroll
			for (uint32_t w = 0; w < 5u; w++)
				if (w < hwords && 4u * w + 4u <= cap)
					*reinterpret_cast<uint32_t *>(fdst + 4u * w) = bswap32(h[w]);
		}
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

// Launch an encode kernel over `grid` blocks (segments).  (A persistent form,
// co-resident workgroups walking the segments, was measured slower: DESIGN.md
// 5.2; passing the kernel arguments on to a device function by reference also
// cost 20 %: the compiler kept them in spilled SGPRs, read back by v_readlane.)
template <typename Kern>
static inline void launch_segments(Kern kern, const KArgs &k, uint32_t grid, size_t lds, hipStream_t s)
{
	hipLaunchKernelGGL(kern, dim3(grid), dim3(EWG), lds, s, k);
}

} // namespace airs
