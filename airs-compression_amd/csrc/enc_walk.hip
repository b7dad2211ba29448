// enc_walk.hip -- MODEL streams in one launch (gfx950).
//
// A batch whose contexts carry a model (secondary MODEL passes, reference
// lib/compress/cmp.c:250-254, update :120-142, applied :304-311) encodes its
// acquisitions in order: frame (c, a+1) reads the model frame (c, a) left.
// The per-acquisition launches of encode_kernel re-read and rewrite that
// model from HBM every step (2 B + 2 B per sample).  Here one launch walks
// every acquisition of every context:
//
//   * workgroup (c, j) owns segment j (4096 samples) of context c's frames
//     and walks a = 0 .. fpc-1; it keeps the model of its samples in
//     registers (8 packed VGPRs per lane) and writes it to the work buffer
//     once, after the last acquisition;
//   * the samples of acquisition a+1 are loaded while acquisition a packs
//     (registers, issued right after phase 1);
//   * waves 0-3 are data waves (16 samples per lane); wave 4 is the control
//     wave: aggregate publish, decoupled look-back over the frame's segments,
//     predecessor tail, frame epilogue (header, checksum, status).  So the
//     data waves never wait on granule loads, whose vmcnt would also wait for
//     their prefetch, and the look-back overlaps their packing;
//   * each frame is its own look-back chain (segments j of frame c*fpc + a).
//
// Pass selection is data-independent here (no fallback, capacity >= worst
// case: the host's asynchronous mode), so every frame's pass follows from the
// context's sequence number at the start of the call (cmp.c:228-248):
// primary when seq == 0 or seq > secondary_iterations.
//
// Per-sample coding (reference encoder.c:303-378): Rice codes come from LDS
// tables, codeword = m + T[idx], length len[idx]:
//   GOLOMB_ZERO  idx = min((m+1) >> k, 17); the escape (q >= 17) is entry 17
//   GOLOMB_MULTI idx = m >> k below the outlier; an escape m >= outlier with
//                d = m - outlier takes idx = 16 + clz(d | 3), whose entry
//                holds golomb(outlier + lvl) shifted over the 2 (lvl+1) bits
//                of d (lvl = floor(log2 d) / 2, 0 for d < 4); the codeword is
//                then m + T as well.  Escapes longer than 32 bits (any lvl
//                once golomb(outlier + lvl) itself nears 32 bits, i.e. an
//                outlier near the upper bound of small g) are put in two
//                pieces, the escape symbol and d.
// Other encoders (UNCOMPRESSED, g not a power of two) take code_from_m.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "enc_common.h"

namespace airs {

// rows of the code tables in LDS (one table per pass)
#define WTAB 48u
// walk_lengths' GOLOMB_MULTI path for waves without an escape (packed, no
// table reads); 0 for A/B builds
#ifndef AIRS_MULTI_FAST
#define AIRS_MULTI_FAST 1
#endif
// The segment walk stores acquisition a in step a + LAG, and keeps LAG + 2
// LDS images: acquisition a + 1 packs into the image stored two steps
// earlier, so no barrier clears the one just stored
#ifndef AIRS_WALK_LAG
#define AIRS_WALK_LAG 1u
#endif
#define AIRS_WALK_NIMG (AIRS_WALK_LAG + 2u)
// counted output stores per data thread and step of the segment walk
// frames per context up to which the segment walk writes its frame epilogues
// after the walk (4 LDS words per frame); 0: in the step loop
#ifndef AIRS_WALK_EPI_MAX
#define AIRS_WALK_EPI_MAX 64u
#endif
#ifndef AIRS_WALK_NQ
#define AIRS_WALK_NQ 1u
#endif

// table entry idx of a pass: {T, len}; see the header comment
template <int ENC>
__device__ __forceinline__ uint2 walk_table_entry(uint32_t idx, const Coder &c)
{
	const uint32_t k = c.k;
	if (ENC == ENC_ZERO)
		return rice_table_entry(idx < 17u ? idx : 17u, k);
	// GOLOMB_MULTI, Rice: g = 2^k
	auto rice_cw = [&](uint32_t v, uint32_t &len) {
		const uint32_t q = v >> k;
		len = q + k + 1u;
		return (((1u << q) - 1u) << (k + 1u)) | (v & (c.g - 1u));
	};
	if (idx < 32u) {
		// T[q] = (2^q - 1) 2^(k+1) - q 2^k (mod 2^32): m + T[q] = golomb(m)
		const uint32_t q = idx;
		const uint32_t t = (q + k + 1u >= 32u ? 0u - (2u << k) : ((1u << (q + k + 1u)) - (2u << k))) - (q << k);
		return make_uint2(t, q + k + 1u);
	}
	const uint32_t tz = idx - 16u; // clz(d | 3) in [16, 30]
	const uint32_t lvl = (31u - tz) >> 1;
	uint32_t len1;
	const uint32_t cw1 = rice_cw(c.outlier + lvl, len1);
	const uint32_t len2 = 2u * (lvl + 1u);
	const uint32_t len = len1 + len2;
	// len > 32: put as two pieces (cw1, then d); T unused
	return make_uint2(len <= 32u ? (cw1 << len2) - c.outlier : cw1, len);
}


// Debug timeline (ablation builds, AIRS_DBG bit 65536): per (workgroup,
// acquisition) 8 slots of the 100 MHz realtime clock: 0 samples in registers,
// 1 after B1, 2 packed, 3 after B2, 4 after B3 (data wave 0); 5 look-back
// done, 6 predecessor tail seen (control wave); 7 HW_ID << 32 | XCC_ID.
// scripts/walk_ts.py summarises it.
__device__ __forceinline__ void wstamp(const WArgs &a, uint32_t acq, uint32_t slot)
{
	if (AIRS_ABLATE && (a.dbg & 65536u) && a.dbgts && (threadIdx.x & 63u) == 0u) {
		uint64_t t;
		asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
		a.dbgts[8u * ((uint64_t)blockIdx.x * a.fpc + acq) + slot] = t;
		if (slot == 0u) {
			uint32_t hw, xcc;
			asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
			asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
			a.dbgts[8u * ((uint64_t)blockIdx.x * a.fpc + acq) + 7u] = ((uint64_t)hw << 32) | xcc;
		}
	}
}

__device__ __forceinline__ void lds_barrier()
{
	// LDS-only barrier: the data waves' prefetch stays in flight across it
	asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Buffer descriptor words of [base, base + bytes): raw buffer, the hardware
// range check drops stores past `bytes`
__device__ __forceinline__ u32x4 rsrc_words(const void *base, uint32_t bytes)
{
	const uint64_t b = (uint64_t)(uintptr_t)base;
	u32x4 r;
	r.x = __builtin_amdgcn_readfirstlane((uint32_t)b);
	r.y = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32) & 0xFFFFu);
	r.z = __builtin_amdgcn_readfirstlane(bytes);
	r.w = 0x00020000u;
	return r;
}

// Output stores the compiler does not count.  The walks issue their sample
// prefetch after the stores of a step; the compiler's wait for the prefetched
// registers then counts only the loads issued after them, instead of falling
// back to vmcnt(0) behind a data-dependent number of stores (which would wait
// for every store and for the prefetch of the step after).
__device__ __forceinline__ void store_b128_nc(u32x4 v, uint32_t byte_off, u32x4 rsrc)
{
	// s_nop 1: a VALU write of the data registers right after a store of more
	// than 64 bits needs wait states, and hipcc does not pad after inline asm
	// (seen: the next address computed into v[18:19] was stored as sample data)
	asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen\n\ts_nop 1" ::"v"(v), "v"(byte_off), "s"(rsrc) : "memory");
}

__device__ __forceinline__ void store_b32_nc(uint32_t v, uint32_t byte_off, u32x4 rsrc)
{
	asm volatile("buffer_store_dword %0, %1, %2, 0 offen" ::"v"(v), "v"(byte_off), "s"(rsrc) : "memory");
}

// one pass's residual-independent coding: table offsets (8 idx per sample,
// 16-bit halves of oq[]), lengths total of the lane; returns the lane's bits
// MF: the GOLOMB_MULTI paths for escape-free waves below (the segment walk;
// the context walk, at 128 VGPRs, measured slower with them: 392-405 against
// 373-379 us on cfg5)
template <int ENC, bool RICE, int NP, bool MF = false>
__device__ __forceinline__ uint32_t walk_lengths(const uint32_t (&mp)[NP], uint32_t (&oq)[NP], const Coder &cd,
						 bool fast, const char *tab)
{
	uint32_t t = 0u;
	if (ENC == ENC_ZERO && RICE && fast) {
		u16x2 acc = (u16x2)(0);
#pragma unroll
		for (uint32_t j = 0; j < NP; j++) {
			const u16x2 v = __builtin_elementwise_add_sat(pk(mp[j]), (u16x2)(1));
			const u16x2 q = v >> (u16x2)((unsigned short)cd.k);
			acc += __builtin_elementwise_min(q, (u16x2)(16));
			oq[j] = unpk(__builtin_elementwise_min(q, (u16x2)(17)) << (u16x2)(3));
		}
		return 2u * NP * (cd.k + 1u) + (unpk(acc) & 0xFFFFu) + (unpk(acc) >> 16);
	}
	if (ENC == ENC_MULTI && RICE) {
		const uint32_t om1 = cd.outlier - 1u;
		// no escape anywhere in the wave (wave-uniform test): every code is
		// unary q = m >> k, then k bits, length q + k + 1; the offsets and
		// the lengths' sum come from packed shifts and adds, no table reads
		// (the sums of NP q per half stay below 2^16: (om1 >> k) NP < 2^16)
		if constexpr (MF) {
			u16x2 mx = (u16x2)(0);
#pragma unroll
			for (uint32_t j = 0; j < NP; j++)
				mx = __builtin_elementwise_max(mx, pk(mp[j]));
			const uint32_t mxu = unpk(mx), mxs = max(mxu & 0xFFFFu, mxu >> 16);
			if (MF && AIRS_MULTI_FAST && (om1 >> cd.k) * NP < 65536u && __ballot(mxs > om1) == 0ull) {
				u16x2 acc = (u16x2)(0);
#pragma unroll
				for (uint32_t j = 0; j < NP; j++) {
					const u16x2 q = pk(mp[j]) >> (u16x2)((unsigned short)cd.k);
					acc += q;
					oq[j] = unpk(q << (u16x2)(3));
				}
				return 2u * NP * (cd.k + 1u) + (unpk(acc) & 0xFFFFu) + (unpk(acc) >> 16);
			}
		}
#pragma unroll
		for (uint32_t j = 0; j < NP; j++) {
			uint32_t o2 = 0u;
#pragma unroll
			for (uint32_t h = 0; h < 2u; h++) {
				const uint32_t m = half16(mp[j], h);
				const uint32_t qo = (m >> cd.k) << 3;
				const uint32_t eo = (((uint32_t)__clz((int)((m - cd.outlier) | 3u))) << 3) + 128u;
				const uint32_t off = m > om1 ? eo : qo;
				o2 |= off << (16u * h);
				t += reinterpret_cast<const uint2 *>(tab + off)->y;
			}
			oq[j] = o2;
		}
		return t;
	}
#pragma unroll
	for (uint32_t j = 0; j < 2u * NP; j++)
		t += len_from_m<ENC, RICE>(half16(mp[j >> 1], j & 1u), cd);
	return t;
}

// pack the lane's 2 NP codewords from bit `excl` of the image
template <int ENC, bool RICE, int NP, bool MF = false>
__device__ __forceinline__ void walk_pack(uint32_t *img, uint32_t excl, const uint32_t (&mp)[NP],
					  const uint32_t (&oq)[NP], const Coder &cd, bool fast, const char *tab)
{
	static_assert(NP % 4 == 0, "batches of 8 samples");
	Packer pk1;
	pk1.init(img, excl);
	if (ENC == ENC_ZERO && RICE && fast) {
#pragma unroll
		for (uint32_t hb = 0; hb < NP / 4u; hb++) { // batches of 8 lookups (pairs of codewords per put)
			uint2 te[8];
#pragma unroll
			for (uint32_t jj = 0; jj < 4u; jj++) {
				const uint32_t j = hb * 4u + jj;
#pragma unroll
				for (uint32_t h = 0; h < 2; h++)
					te[2 * jj + h] = *reinterpret_cast<const uint2 *>(tab + half16(oq[j], h));
			}
			uint32_t mxl = 0u;
#pragma unroll
			for (uint32_t i = 0; i < 8u; i += 2)
				mxl = max(mxl, te[i].y + te[i + 1].y);
			if (__ballot(mxl > 32u) == 0ull) {
#pragma unroll
				for (uint32_t i = 0; i < 8u; i += 2) {
					const uint32_t j = hb * 8u + i;
					const uint32_t cwa = (mp[j >> 1] & 0xFFFFu) + te[i].x;
					const uint32_t cwb = (mp[j >> 1] >> 16) + te[i + 1].x;
					pk1.put((cwa << te[i + 1].y) | cwb, te[i].y + te[i + 1].y);
				}
			} else {
#pragma unroll
				for (uint32_t i = 0; i < 8u; i += 2) {
					const uint32_t j = hb * 8u + i;
					pk1.put((mp[j >> 1] & 0xFFFFu) + te[i].x, te[i].y);
					pk1.put((mp[j >> 1] >> 16) + te[i + 1].x, te[i + 1].y);
				}
			}
		}
	} else if (ENC == ENC_MULTI && RICE) {
		// batches of 8 lookups issued before their puts: one at a time, each
		// lookup waited for the LDS (and the puts before it) on its own,
		// 16 serial LDS round trips per lane
#pragma unroll
		for (uint32_t hb = 0; hb < NP / 4u; hb++) {
			uint2 te[8];
#pragma unroll
			for (uint32_t i = 0; i < 8u; i++) {
				const uint32_t j = hb * 8u + i;
				te[i] = *reinterpret_cast<const uint2 *>(tab + half16(oq[j >> 1], j & 1u));
			}
			// every pair of the batch fits one put (the wave's short codes, as
			// in the ZERO path): half the puts
			uint32_t mxl = 0u;
			if constexpr (MF) {
#pragma unroll
				for (uint32_t i = 0; i < 8u; i += 2)
					mxl = max(mxl, te[i].y + te[i + 1].y);
			}
			if (MF && AIRS_MULTI_FAST && __ballot(mxl > 32u) == 0ull) {
#pragma unroll
				for (uint32_t i = 0; i < 8u; i += 2) {
					const uint32_t j = hb * 8u + i;
					const uint32_t cwa = (mp[j >> 1] & 0xFFFFu) + te[i].x;
					const uint32_t cwb = (mp[j >> 1] >> 16) + te[i + 1].x;
					pk1.put((cwa << te[i + 1].y) | cwb, te[i].y + te[i + 1].y);
				}
				continue;
			}
#pragma unroll
			for (uint32_t i = 0; i < 8u; i++) {
				const uint32_t j = hb * 8u + i;
				const uint32_t m = half16(mp[j >> 1], j & 1u);
				const uint2 e = te[i];
				if (e.y <= 32u) {
					pk1.put(m + e.x, e.y);
				} else { // escape longer than 32 bits: golomb(outlier + lvl), then d in 2 (lvl + 1) bits
					const uint32_t off = half16(oq[j >> 1], j & 1u);
					const uint32_t len2 = 2u * (((31u - ((off >> 3) - 16u)) >> 1) + 1u);
					pk1.put(e.x, e.y - len2);
					pk1.put(m - cd.outlier, len2);
				}
			}
		}
	} else {
#pragma unroll
		for (uint32_t j = 0; j < 2u * NP; j++) {
			uint32_t c1, l1, c2, l2;
			code_from_m<ENC, RICE>(half16(mp[j >> 1], j & 1u), cd, c1, l1, c2, l2);
			pk1.put(c1, l1);
			if (ENC == ENC_MULTI)
				pk1.put(c2, l2);
		}
	}
	pk1.flush();
}

// the frame's first payload dword shares header bytes 20-21 (outlier low half)
__device__ __forceinline__ uint32_t hdr_bits(int pre, int enc)
{
	return (pre == PRE_NONE && enc == ENC_RAW) ? 128u : 176u;
}

// Four data waves of E samples per lane (16 or 8) and one control wave: a
// segment is 256 E samples.  E = 8 doubles the workgroups (and the waves) of
// a batch, for batches of few contexts (configs[4]'s 32 streams per GPU at
// N = 8: 1024 workgroups instead of 512, 4 data waves per SIMD instead of 2):
// a step is latency-bound per wave (LDS lookups and puts in the packing), so
// twice the waves with half the samples each shorten it.
template <int W, int PRE_P, int ENC_P, bool RICE_P, int ENC_S, bool RICE_S, int E>
__global__ __launch_bounds__(320) void walk_kernel(WArgs a)
{
	static_assert(E == 16 || E == 8, "16 or 8 samples per lane");
	constexpr uint32_t DW = 4u;
	constexpr uint32_t RW = E * W / 16u; // uint4 per lane
	constexpr uint32_t NT = 64u * (DW + 1u), ND = 64u * DW; // threads, data threads
	constexpr uint32_t SEGW = ND * E;                        // samples per segment
	extern __shared__ __attribute__((aligned(16))) uint32_t L_img[];
	__shared__ uint32_t s_wsum[DW];
	__shared__ uint32_t s_ctl[4];
	__shared__ __attribute__((aligned(16))) uint2 s_tab[2][WTAB];

	const uint32_t tid = threadIdx.x, lane = tid & 63u;
	const uint32_t wid = __builtin_amdgcn_readfirstlane(tid >> 6);
	const bool data = wid < DW;
	// logical block index from a ticket taken at start: every
	// workgroup with a smaller index has started (is resident or done), so a
	// look-back only ever waits on a workgroup that is running, whatever order
	// the XCDs dispatch in.  A grid that the CUs hold at once (a.direct,
	// host-checked occupancy) takes the block index instead: every workgroup
	// is running, and 1024 tickets on one counter spread the workgroups'
	// start over ~13 us (cfg5s8 with 2048-sample segments)
	// (A direct launch does not touch the counter at all: even an atomic
	// without return is older than the workgroup's first sample loads, and
	// vmcnt completes in order, so their wait included the counter's queue.)
	uint32_t lb = blockIdx.x;
	if (!a.direct) {
		if (tid == 0u)
			s_ctl[3] = atomicAdd(a.ticket + AIRS_WALK_TICKET, 1u) - a.ticket_base;
		__syncthreads();
		lb = __builtin_amdgcn_readfirstlane(s_ctl[3]);
	}
	// Dispatch generation (direct launches): the CUs take the grid one
	// workgroup each per generation, so block b is its CU's (b / CUs)-th.  At
	// equal priority the oldest waves issue first: the CU's first workgroup
	// finished its walk in 44 us and its fourth in 62 (cfg5s8), the CU nearly
	// empty at the end; a fixed priority by generation only inverts that.  The
	// data waves rotate their priority by step and generation instead (below).
	const uint32_t gen = (a.direct && a.cus) ? blockIdx.x / a.cus : 0u;
	auto rotate_prio = [&](uint32_t acq) {
		if (!(a.direct && a.cus))
			return;
		const uint32_t pr = (acq + gen) & 3u;
		if (pr == 0u)
			__builtin_amdgcn_s_setprio(0);
		else if (pr == 1u)
			__builtin_amdgcn_s_setprio(1);
		else if (pr == 2u)
			__builtin_amdgcn_s_setprio(2);
		else
			__builtin_amdgcn_s_setprio(3);
	};
	const uint32_t c = lb / a.spf, j = lb - c * a.spf;
	const bool is_first = j == 0u, is_last = j + 1u == a.spf;
	const uint32_t n = a.n;
	const uint32_t first = j * SEGW + (data ? tid : 0u) * E; // lane's first sample
	uint16_t *mbase = reinterpret_cast<uint16_t *>(a.model_ptrs ? (uint8_t *)(uintptr_t)a.model_ptrs[c]
								    : a.model + (uint64_t)c * a.model_stride);
	// NIMG images (a.img_words each, after a 4-word pad): acquisition a packs
	// into image a % NIMG and is stored in the next step, once its frame
	// offset is known.  With three, the image acquisition a + 1 packs into was
	// stored two steps earlier, so it is cleared without a third barrier
	constexpr uint32_t LAG = AIRS_WALK_LAG;
	constexpr uint32_t NIMG = AIRS_WALK_NIMG;
	static_assert((LAG == 1u || LAG == 2u) && NIMG == LAG + 2u, "images: the lag plus two");
	auto img_at = [&](uint32_t q) { return L_img + 4u + (q % NIMG) * (a.img_words + 4u); };

	const Coder cp = make_coder<ENC_P>(ENC_P == ENC_RAW ? 1u : a.g_p, a.outl_p);
	const Coder cs = make_coder<ENC_S>(ENC_S == ENC_RAW ? 1u : a.g_s, a.outl_s);
	const bool fast_p = RICE_P && (ENC_P == ENC_MULTI || (ENC_P == ENC_ZERO && cp.k <= 11u));
	const bool fast_s = RICE_S && (ENC_S == ENC_MULTI || (ENC_S == ENC_ZERO && cs.k <= 11u));
	if (tid < WTAB) {
		if (fast_p)
			s_tab[0][tid] = walk_table_entry<ENC_P>(tid, cp);
		if (fast_s)
			s_tab[1][tid] = walk_table_entry<ENC_S>(tid, cs);
	}
	for (uint32_t i = tid; i < NIMG * (a.img_words + 4u) + 4u; i += NT)
		L_img[i] = 0u;

	const uint32_t seq0 = a.seq0s ? a.seq0s[c] : a.seq0;
	// Samples and model are kept "flipped" (i16: the sign bit of every half
	// inverted, u16: as they are), so that both sample types take the model
	// update of zero-extended halves (model_update_zx); residuals are
	// differences and do not change
	const uint32_t flip = a.is_unsigned ? 0u : 0x80008000u;
	// the model of this lane's 16 samples, packed pairs
	uint32_t mdl[E / 2];
#pragma unroll
	for (uint32_t q = 0; q < E / 2; q++)
		mdl[q] = 0u;
	if (data && seq0 != 0u && seq0 <= a.iters) { // the first frame is a secondary pass
		const uint4 *mp4 = reinterpret_cast<const uint4 *>(mbase + first);
#pragma unroll
		for (uint32_t q = 0; q < E / 8; q++) {
			const uint4 v = mp4[q];
			mdl[4 * q] = v.x ^ flip;
			mdl[4 * q + 1] = v.y ^ flip;
			mdl[4 * q + 2] = v.z ^ flip;
			mdl[4 * q + 3] = v.w ^ flip;
		}
	}
	// prefetch of acquisition 0
	uint4 rn[RW];
	uint32_t pn = 0u;
	// unconditional loads, every data lane (the sample before the lane's first
	// matters to lane 0 only; its low half is taken at the use): a load under
	// a condition into registers that stay live makes the compiler wait for
	// it, and for the prefetch issued with it, right after the issue
	auto issue = [&](uint32_t acq) {
		const uint8_t *fs = a.src + (uint64_t)(c * a.fpc + acq) * a.src_stride;
		const uint4 *p = reinterpret_cast<const uint4 *>(fs + (size_t)first * W);
#pragma unroll
		for (uint32_t q = 0; q < RW; q++)
			rn[q] = p[q];
		if (PRE_P == PRE_DIFF) {
			const uint32_t ip = first ? first - 1u : 0u;
			pn = W == 2 ? (uint32_t)reinterpret_cast<const uint16_t *>(fs)[ip]
				    : reinterpret_cast<const uint32_t *>(fs)[ip];
		}
	};
	if (data)
		issue(0u);
	__syncthreads(); // tables and the zeroed images

	const char *tab_p = reinterpret_cast<const char *>(s_tab[0]);
	const char *tab_s = reinterpret_cast<const char *>(s_tab[1]);
	// Step `acq` codes acquisition acq (acq < fpc) and stores acquisition
	// acq - LAG (acq >= LAG).  The look-back of acquisition acq - LAG runs in
	// step acq: every segment published its aggregate and tail for it LAG
	// steps earlier, so it is one granule round trip (look-back window and
	// tail together, issued at the end of the step before), and it never
	// waits on a chain of predecessors; with LAG = 2 it has a whole step to
	// return, so the control wave is not what the step's B2 waits for.
	//
	// The data waves and the control wave run separate copies of the step loop
	// (same barriers, B1 and B2 per step).  In one shared loop the compiler's
	// wait analysis merged the control wave's granule loads into the data
	// waves' paths and made the data waves wait for everything outstanding
	// (their own sample prefetch included) before the store.  The data waves'
	// output stores are a fixed number per step (past the capacity when there
	// is nothing to store: dropped by the buffer range check), so the wait for
	// the next step's samples counts exactly the stores issued after them.
	uint32_t sq = seq0;
	if (data) {
		// the first samples and the model in registers before the loop: the
		// loop head then has the same outstanding operations on entry as from
		// its back edge (the step's stores), and the compiler's wait there
		// need not cover them (vmcnt(0), expcnt and lgkmcnt left alone)
		__builtin_amdgcn_s_waitcnt(0x0F70);
		uint32_t A1 = 0u, A2 = 0u, A3 = 0u; // the bit totals of acquisitions acq - 1, acq - 2, acq - 3
		// quads of one image per data thread, at most (48-bit codewords)
		// counted 16-byte stores per thread and step: one covers segments of up
		// to 16 bits per sample (cfg5's are ~7); the quads past it (noisy
		// segments) go out uncounted (the fixed-count form with room for 48-bit
		// codes cost ~6 VALU instructions per sample at 8 samples per lane)
		constexpr uint32_t NQ = AIRS_WALK_NQ;
		for (uint32_t acq = 0; acq < a.fpc + LAG; acq++) {
			const bool have = acq < a.fpc, prev = acq >= LAG;
			const uint32_t f = c * a.fpc + acq;
			const bool prim = sq == 0u || sq > a.iters; // cmp.c:228-248
			if (have)
				sq = prim ? 1u : sq + 1u;
			rotate_prio(acq);
			uint32_t *const img = img_at(acq);
			uint32_t *const imgp = img_at(acq + NIMG - LAG); // acquisition acq - LAG
			uint32_t mp[E / 2], oq[E / 2];
			uint32_t T = 0u, excl = 0u;
			if (have) {
				// ---- phase 1: samples, residuals, model update, lengths ----------
				uint32_t w[E / 2];
				if (W == 2) {
#pragma unroll
					for (uint32_t q = 0; q < RW; q++) {
						w[4 * q] = rn[q].x ^ flip;
						w[4 * q + 1] = rn[q].y ^ flip;
						w[4 * q + 2] = rn[q].z ^ flip;
						w[4 * q + 3] = rn[q].w ^ flip;
					}
				} else {
#pragma unroll
					for (uint32_t q = 0; q < RW; q++) {
						w[2 * q] = __builtin_amdgcn_perm(rn[q].y, rn[q].x, 0x05040100u) ^ flip;
						w[2 * q + 1] = __builtin_amdgcn_perm(rn[q].w, rn[q].z, 0x05040100u) ^ flip;
					}
				}
				if (wid == 0u)
					wstamp(a, acq, 0u);
				const uint32_t prevs = first ? pn & 0xFFFFu : 0u;
				issue(acq + 1u < a.fpc ? acq + 1u : acq); // lands while this acquisition packs (the last reloads)
				if (prim) {
					uint32_t wprev = 0u;
					if (PRE_P == PRE_DIFF) {
						wprev = __shfl_up(w[E / 2 - 1], 1, 64);
						if (lane == 0u)
							wprev = (prevs << 16) ^ flip;
					}
#pragma unroll
					for (uint32_t q = 0; q < E / 2; q++) {
						uint32_t u = w[q] ^ flip; // NONE: the sample itself
						if (PRE_P == PRE_DIFF)
							u = unpk(pk(w[q]) - pk(__builtin_amdgcn_alignbit(w[q], q ? w[q - 1] : wprev, 16)));
						mp[q] = ENC_P == ENC_RAW ? u : zigzag_pk(u);
						mdl[q] = w[q]; // cmp.c:305-306: the model takes the samples
					}
					T = walk_lengths<ENC_P, RICE_P, E / 2, true>(mp, oq, cp, fast_p, tab_p);
				} else {
					const int32_t r1 = 16 - (int32_t)a.model_rate;
#pragma unroll
					for (uint32_t q = 0; q < E / 2; q++) {
						const uint32_t u = unpk(pk(w[q]) - pk(mdl[q])); // preprocess.c:406-411
						mp[q] = ENC_S == ENC_RAW ? u : zigzag_pk(u);
						mdl[q] = model_update_zx(w[q], mdl[q], r1); // cmp.c:132-142
					}
					T = walk_lengths<ENC_S, RICE_S, E / 2, true>(mp, oq, cs, fast_s, tab_s);
				}
#pragma unroll
				for (uint32_t q = 0; q < E / 2; q++)
					asm volatile("" : "+v"(mp[q]), "+v"(oq[q]));
				const uint32_t inc = wave_incl_scan(T);
				if (lane == 63u)
					s_wsum[wid] = inc;
				excl = inc - T;
			}
			lds_barrier(); // B1: wave totals
			uint32_t Asum = 0u, wpre = 0u;
#pragma unroll
			for (uint32_t w = 0; w < DW; w++) {
				const uint32_t v = s_wsum[w];
				wpre += w < wid ? v : 0u;
				Asum += v;
			}
			const uint32_t A = have ? __builtin_amdgcn_readfirstlane(Asum) : 0u;
			if (wid == 0u)
				wstamp(a, acq < a.fpc ? acq : a.fpc - 1u, 1u);
			if (have) {
				excl += wpre;
				// ---- pack into this acquisition's image -----------------------------
				if (prim)
					walk_pack<ENC_P, RICE_P, E / 2, true>(img, excl, mp, oq, cp, fast_p, tab_p);
				else
					walk_pack<ENC_S, RICE_S, E / 2, true>(img, excl, mp, oq, cs, fast_s, tab_s);
				if (wid == DW - 1u && !is_last) {
					// the segment's last 32 bits (wave 3's own lanes wrote them) for
					// the successor's first word (read by it one step later)
					asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
					const uint32_t s0 = A - 32u, qw = s0 >> 5, sh = s0 & 31u;
					const uint32_t tl = sh ? (img[qw] << sh) | (img[qw + 1u] >> (32u - sh)) : img[qw];
					if (lane == 0u)
						gran_store(&a.tail[(uint64_t)f * a.spf + j], ((uint64_t)a.epoch << 32) | tl);
				}
				if (wid == 0u)
					wstamp(a, acq, 2u);
			}
			lds_barrier(); // B2: this step's image packed; the previous step's offset and predecessor bits
			// ---- store acquisition acq - LAG: funnel shift to the frame bit
			// offset, big-endian; NQ + 1 stores per thread in every step -------
			{
				const uint32_t A_st = LAG == 2u ? A2 : A1;
				const uint32_t P = __builtin_amdgcn_readfirstlane(s_ctl[0]);
				const uint32_t pred = __builtin_amdgcn_readfirstlane(s_ctl[1]);
				const uint32_t r = P & 31u, g0 = P >> 5;
				const uint32_t endbit = P + A_st;
				const uint32_t J = ((endbit - 1u) >> 5) - g0; // last word touched
				const uint32_t nfull = prev ? ((endbit & 31u) == 0u ? J + 1u : J) : 0u;
				uint8_t *fdst = a.dst + (uint64_t)(prev ? f - LAG : f) * a.dst_stride;
				const __amdgpu_buffer_rsrc_t dst_rsrc =
					__builtin_amdgcn_make_buffer_rsrc(fdst, 0, (int)(a.cap & ~3u), 0x00020000);
				const lds_u32 *Ll = reinterpret_cast<const lds_u32 *>((uintptr_t)imgp);
				const uint32_t nquad = nfull >> 2;
#pragma unroll
				for (uint32_t i = 0; i < NQ; i++) {
					const uint32_t p = tid + i * ND;
					const bool in = p < nquad;
					const uint32_t jw = in ? 4u * p : 0u;
					const u32x4 wv = *reinterpret_cast<const __attribute__((address_space(3))) u32x4 *>(Ll + jw);
					const uint32_t hi = jw ? Ll[jw - 1u] : pred;
					u32x4 o;
					o.x = bswap32(__builtin_amdgcn_alignbit(hi, wv.x, r));
					o.y = bswap32(__builtin_amdgcn_alignbit(wv.x, wv.y, r));
					o.z = bswap32(__builtin_amdgcn_alignbit(wv.y, wv.z, r));
					o.w = bswap32(__builtin_amdgcn_alignbit(wv.z, wv.w, r));
					// past the buffer range when there is nothing to store: dropped
					__builtin_amdgcn_raw_buffer_store_b128(o, dst_rsrc, in ? (int)(4u * (g0 + jw)) : INT32_MIN, 0, 0);
				}
				const uint32_t rr = (tid - nquad) & (ND - 1u);
				const bool part = rr < (nfull & 3u);
				const uint32_t jw = part ? 4u * nquad + rr : 0u;
				const uint32_t hi = jw ? Ll[jw - 1u] : pred;
				const uint32_t v = __builtin_amdgcn_alignbit(hi, Ll[jw], r);
				__builtin_amdgcn_raw_buffer_store_b32(bswap32(v), dst_rsrc, part ? (int)(4u * (g0 + jw)) : INT32_MIN, 0,
								      0);
				if (nquad > NQ * ND) { // the rest, uncounted (walk_ctx_kernel's stores)
					const u32x4 rs4 = rsrc_words(fdst, a.cap & ~3u);
					for (uint32_t p = tid + NQ * ND; p < nquad; p += ND) {
						const uint32_t jq = 4u * p;
						const u32x4 wv =
							*reinterpret_cast<const __attribute__((address_space(3))) u32x4 *>(Ll + jq);
						const uint32_t hq = Ll[jq - 1u];
						u32x4 o;
						o.x = bswap32(__builtin_amdgcn_alignbit(hq, wv.x, r));
						o.y = bswap32(__builtin_amdgcn_alignbit(wv.x, wv.y, r));
						o.z = bswap32(__builtin_amdgcn_alignbit(wv.y, wv.z, r));
						o.w = bswap32(__builtin_amdgcn_alignbit(wv.z, wv.w, r));
						store_b128_nc(o, 4u * (g0 + jq), rs4);
					}
				}
				if (prev && wid == 0u)
					wstamp(a, acq - LAG, 4u);
			}
			// acquisition acq + 1 packs into the image of acquisition
			// acq + 1 - NIMG = acq - LAG - 1, stored in step acq - 1: every wave
			// finished that store before this step's B1.  Clear it (visible to
			// that packing after the next B1)
			if (acq >= LAG + 1u && acq + 1u < a.fpc) {
				uint32_t *const imgn = img_at(acq + 1u);
				const uint32_t nw = ((LAG == 2u ? A3 : A2) + 63u) >> 5;
				for (uint32_t i = tid; i < nw; i += ND)
					imgn[i] = 0u;
			}
			A3 = A2;
			A2 = A1;
			A1 = A;
		}
	} else {
		// ---- the control wave: aggregates, look-backs, predecessor tails,
		// frame epilogues ----------------------------------------------------
		// acquisitions acq - 1 and acq - 2: bit total, header bits, header
		// sequence number, primary pass
		uint32_t A1 = 0u, HB1 = 0u, hseq1 = 0u, A2 = 0u, HB2 = 0u, hseq2 = 0u;
		bool prim1 = false, prim2 = false;
		// the first look-back round of the acquisition to store next step and
		// its predecessor tail, issued at the end of the step before, evaluated
		// after B1
		uint64_t gv0 = 0ull, tv0 = 0ull;
		// The frame epilogue's stores (header words, final bytes, checksum,
		// status: partial cache lines) cost the last segment's control wave
		// ~5 us per cfg5s8 launch inside the step loop (the compiler's waits
		// for the next look-back loads covered them).  With at most
		// AIRS_WALK_EPI_MAX frames per context they are kept in LDS (four words
		// per frame) and written after the walk, one frame per lane.
		const bool defer = a.fpc <= AIRS_WALK_EPI_MAX;
		uint32_t *const epi = L_img + 4u + NIMG * (a.img_words + 4u);
		// frame ai of this context: payload bytes, final word (written when
		// nbytes > 0) at byte offset fwoff, meta = header sequence number |
		// primary << 8 | 22-byte header << 9 | nbytes << 16
		auto frame_epilogue = [&](uint32_t ai, uint32_t payload_bytes, uint32_t v, uint32_t fwoff, uint32_t meta) {
			const uint32_t fp = c * a.fpc + ai;
			uint8_t *fdst = a.dst + (uint64_t)fp * a.dst_stride;
			const uint32_t nbytes = meta >> 16;
			for (uint32_t b = 0; b < nbytes; b++)
				if (fwoff + b < a.cap)
					fdst[fwoff + b] = (uint8_t)(v >> (24u - 8u * b));
			const uint32_t size = payload_bytes + (a.checksum ? 4u : 0u);
			if (a.checksum) {
				const uint32_t ck = a.checksums[fp];
				for (uint32_t b = 0; b < 4u; b++)
					if (payload_bytes + b < a.cap)
						fdst[payload_bytes + b] = (uint8_t)(ck >> (24u - 8u * b));
			}
			const uint64_t id = a.ids ? a.ids[fp] : a.id_base + (uint64_t)c * a.id_cstep + (uint64_t)ai * a.id_astep;
			const uint32_t hs = meta & 0xFFu;
			uint32_t h[5];
			if (meta & 0x100u)
				header_words(h, size, 2u * n, id, hs, PRE_P, a.checksum ? 1u : 0u, ENC_P, 0u,
					     ENC_P == ENC_RAW ? 0u : cp.g, ENC_P == ENC_RAW ? 0u : cp.outlier);
			else
				header_words(h, size, 2u * n, id, hs, PRE_MODEL, a.checksum ? 1u : 0u, ENC_S, a.model_rate,
					     ENC_S == ENC_RAW ? 0u : cs.g, ENC_S == ENC_RAW ? 0u : cs.outlier);
			const uint32_t hwords = (meta & 0x200u) ? 5u : 4u;
			for (uint32_t wq = 0; wq < hwords; wq++)
				if (4u * wq + 4u <= a.cap)
					*reinterpret_cast<uint32_t *>(fdst + 4u * wq) = bswap32(h[wq]);
			a.status[fp] = size > a.cap ? ERRV(E_DST_TOO_SMALL) : size > 0xFFFFFFu ? ERRV(E_HDR_CMP_SIZE_TOO_LARGE) : size;
		};
		for (uint32_t acq = 0; acq < a.fpc + LAG; acq++) {
			const bool have = acq < a.fpc, prev = acq >= LAG;
			const uint32_t f = c * a.fpc + acq;
			const bool prim = sq == 0u || sq > a.iters; // cmp.c:228-248
			const uint32_t hseq = prim ? 0u : sq;
			if (have)
				sq = prim ? 1u : sq + 1u;
			const uint32_t HB = prim ? hdr_bits(PRE_P, ENC_P) : hdr_bits(PRE_MODEL, ENC_S);
			lds_barrier(); // B1: wave totals
			uint32_t Asum = 0u;
#pragma unroll
			for (uint32_t w = 0; w < DW; w++)
				Asum += s_wsum[w];
			const uint32_t A = have ? __builtin_amdgcn_readfirstlane(Asum) : 0u;
			if (have && lane == 0u) {
				const uint64_t tag = ((uint64_t)a.epoch << 1) | (is_first ? 1u : 0u);
				gran_store(&a.agg[(uint64_t)f * a.spf + j], (tag << 32) | (is_first ? HB + A : A));
			}
			const uint32_t A_st = LAG == 2u ? A2 : A1, HB_st = LAG == 2u ? HB2 : HB1;
			const uint32_t hseq_st = LAG == 2u ? hseq2 : hseq1;
			const bool prim_st = LAG == 2u ? prim2 : prim1;
			uint32_t P = HB_st, pred = 0u;
			if (prev) {
				const uint64_t gseg = (uint64_t)(f - LAG) * a.spf + j;
				if (is_first) {
					const uint32_t enc = prim_st ? ENC_P : ENC_S;
					pred = (enc != ENC_RAW) ? ((prim_st ? cp.outlier : cs.outlier) & 0xFFFFu) : 0u;
				} else {
					const uint64_t first_seg = gseg - j;
					uint32_t sum = 0u, spins = 0u;
					int64_t jj = (int64_t)gseg - 1;
					uint64_t gv = gv0;
					for (;;) {
						const int64_t idx = jj - (int64_t)lane;
						const bool inr = idx >= (int64_t)first_seg;
						const uint32_t tag = (uint32_t)(gv >> 32);
						const bool valid = inr && (tag >> 1) == a.epoch;
						const bool incl = valid && (tag & 1u);
						const uint64_t incl_m = __ballot(incl);
						const uint64_t bad_m = __ballot(inr && !valid);
						const uint32_t fi = incl_m ? (uint32_t)__ffsll((unsigned long long)incl_m) - 1u : 64u;
						const uint64_t need = fi >= 63u ? ~0ull : ((2ull << fi) - 1ull);
						if (bad_m & need) { // a needed predecessor has not published yet
							if (++spins > AIRS_SPIN_LIMIT) {
								if (lane == 0)
									atomicAdd(a.ticket + AIRS_FAULT_WORD, 1u);
								break;
							}
							__builtin_amdgcn_s_sleep(1);
							gv = inr ? gran_load(&a.agg[idx]) : 0ull;
							continue;
						}
						sum += wave_sum((inr && lane <= fi) ? (uint32_t)gv : 0u);
						if (incl_m)
							break;
						jj -= 64;
						gv = jj - (int64_t)lane >= (int64_t)first_seg ? gran_load(&a.agg[jj - (int64_t)lane]) : 0ull;
					}
					P = sum;
					if (lane == 0u)
						gran_store(&a.agg[gseg], ((((uint64_t)a.epoch << 1) | 1u) << 32) | (P + A_st));
					wstamp(a, acq - LAG, 5u);
					// the predecessor's last 32 bits (published after its packing)
					uint64_t tv = tv0;
					if (lane == 0u) {
						uint32_t sp = 0u;
						for (; (uint32_t)(tv >> 32) != a.epoch; tv = gran_load(&a.tail[gseg - 1u])) {
							if (++sp > AIRS_SPIN_LIMIT) {
								atomicAdd(a.ticket + AIRS_FAULT_WORD, 1u);
								break;
							}
							__builtin_amdgcn_s_sleep(1);
						}
					}
					pred = (uint32_t)__shfl(tv, 0, 64);
					wstamp(a, acq - LAG, 6u);
				}
				if (lane == 0u) {
					s_ctl[0] = P;
					s_ctl[1] = pred;
				}
			}
			lds_barrier(); // B2
			if (prev && is_last && lane == 0u) {
				// ---- frame epilogue (cmp.c:314-334): the final word, kept for
				// the end of the walk (or written now, frame_epilogue) --------------
				uint32_t *const imgp = img_at(acq + NIMG - LAG);
				const uint32_t r = P & 31u, g0 = P >> 5;
				const uint32_t endbit = P + A_st;
				const uint32_t J = ((endbit - 1u) >> 5) - g0; // last word touched
				const uint32_t nfull = (endbit & 31u) == 0u ? J + 1u : J;
				uint32_t v = 0u, nbytes = 0u;
				if (nfull == J) { // zero-padded final bytes (bitstream_flush)
					const uint32_t hi = J ? imgp[J - 1u] : pred;
					v = __builtin_amdgcn_alignbit(hi, imgp[J], r);
					nbytes = ((endbit & 31u) + 7u) >> 3;
				}
				const uint32_t meta = hseq_st | (prim_st ? 0x100u : 0u) | (HB_st == 176u ? 0x200u : 0u) | nbytes << 16;
				if (defer) {
					uint32_t *const rec = epi + 4u * (acq - LAG);
					rec[0] = (endbit + 7u) >> 3;
					rec[1] = v;
					rec[2] = 4u * (g0 + J);
					rec[3] = meta;
				} else {
					frame_epilogue(acq - LAG, (endbit + 7u) >> 3, v, 4u * (g0 + J), meta);
				}
			}
			if (acq + 1u >= LAG && acq + 1u - LAG < a.fpc && !is_first) {
				// the look-back of acquisition acq + 1 - LAG (next step)
				const uint64_t gseg = (uint64_t)(c * a.fpc + acq + 1u - LAG) * a.spf + j;
				const int64_t idx = (int64_t)gseg - 1 - (int64_t)lane;
				tv0 = lane == 0u ? gran_load(&a.tail[gseg - 1u]) : 0ull;
				gv0 = idx >= (int64_t)(gseg - j) ? gran_load(&a.agg[idx]) : 0ull;
			}
			A2 = A1;
			HB2 = HB1;
			hseq2 = hseq1;
			prim2 = prim1;
			A1 = A;
			HB1 = HB;
			hseq1 = hseq;
			prim1 = prim;
		}
		if (defer && is_last) {
			// the epilogues kept in LDS (written by this wave's lane 0)
			for (uint32_t ai = lane; ai < a.fpc; ai += 64u) {
				const uint32_t *const rec = epi + 4u * ai;
				frame_epilogue(ai, rec[0], rec[1], rec[2], rec[3]);
			}
		}
	}
	// the model after the last acquisition, to the work buffer (cmp.c:304-311)
	if (data) {
		uint4 *mo = reinterpret_cast<uint4 *>(mbase + first);
#pragma unroll
		for (uint32_t q = 0; q < E / 8; q++)
			mo[q] = make_uint4(mdl[4 * q] ^ flip, mdl[4 * q + 1] ^ flip, mdl[4 * q + 2] ^ flip, mdl[4 * q + 3] ^ flip);
	}
}

// ---------------------------------------------------------------------
// One context per workgroup (walk_ctx_kernel): 1024 threads walk every
// acquisition of ONE context, CH chunks of 16384 samples per frame (frames of
// CH * 16384 samples).  A frame never leaves the workgroup, so the chunks'
// bit offsets are a running sum inside it: no look-back, no granule, no
// handoff between workgroups (the segment walk above pays two handoffs per
// acquisition step, which serialise the 16 segments of a context).
//   * lane t owns samples [16t, 16t+16) of each chunk and keeps their model
//     in registers (CH x 8 packed VGPRs);
//   * the samples of the chunk two steps ahead are loaded while a chunk is
//     coded (two register sets);
//   * each chunk is packed into one of two LDS images at its frame bit offset
//     mod 32, so image word i IS frame word (P >> 5) + i: the store needs no
//     funnel shift; the chunk's partial last word is carried into the next
//     chunk's image word 0 (the frame's first chunk starts with header bytes
//     20-21);
//   * two barriers per chunk: wave totals (B1), packed image (B2).
// ---------------------------------------------------------------------
#define CW_THREADS 1024u
// the context walk's counted stores per thread and chunk (cw_chunk NQ): 0,
// all uncounted.  The kernel sits at 128 VGPRs; counted stores (2 per thread,
// or 5, enough for any chunk) spilled to scratch
#ifndef CW_NQ
#define CW_NQ 0u
#endif
#define CW_WAVES (CW_THREADS / 64u)
#define CW_CHUNK (CW_THREADS * EPT)
// register sets of prefetched samples (1: the next chunk is loaded while one
// is coded; 2: the one after it as well)
#ifndef CW_DEPTH
#define CW_DEPTH 1
#endif

// the 16 samples of this lane from a register set, as packed flipped pairs
template <int W>
__device__ __forceinline__ void cw_pairs(const uint4 (&r)[EPT * W / 16u], uint32_t flip, uint32_t (&w)[EPT / 2])
{
	if (W == 2) {
#pragma unroll
		for (uint32_t q = 0; q < EPT / 8; q++) {
			w[4 * q] = r[q].x ^ flip;
			w[4 * q + 1] = r[q].y ^ flip;
			w[4 * q + 2] = r[q].z ^ flip;
			w[4 * q + 3] = r[q].w ^ flip;
		}
	} else {
#pragma unroll
		for (uint32_t q = 0; q < EPT / 4; q++) {
			w[2 * q] = __builtin_amdgcn_perm(r[q].y, r[q].x, 0x05040100u) ^ flip;
			w[2 * q + 1] = __builtin_amdgcn_perm(r[q].w, r[q].z, 0x05040100u) ^ flip;
		}
	}
}

// NONE/DIFF residuals of a flipped pair sequence (ZigZag unless UNCOMPRESSED)
template <int PRE, int ENC>
__device__ __forceinline__ void cw_primary(const uint32_t (&w)[EPT / 2], uint32_t prevs, uint32_t flip, uint32_t lane,
					   uint32_t (&mp)[EPT / 2])
{
	uint32_t wprev = 0u;
	if (PRE == PRE_DIFF) {
		wprev = __shfl_up(w[EPT / 2 - 1], 1, 64);
		if (lane == 0u)
			wprev = (prevs << 16) ^ flip;
	}
#pragma unroll
	for (uint32_t q = 0; q < EPT / 2; q++) {
		uint32_t u = w[q] ^ flip;
		if (PRE == PRE_DIFF)
			u = unpk(pk(w[q]) - pk(__builtin_amdgcn_alignbit(w[q], q ? w[q - 1] : wprev, 16)));
		mp[q] = ENC == ENC_RAW ? u : zigzag_pk(u);
	}
}

// Chunk state of a workgroup walk: the chunk's frame bit offset P, the bits
// before it in its first word (carry), image words the previous chunk used
struct CwState {
	uint32_t P, carry, used_prev;
};

// One chunk after its lengths: block scan (B1), packing at the frame bit
// offset mod 32 into img (the carry ORed into word 0), B2, store of the whole
// words (frame word (P >> 5) + i, big-endian), carry of the partial last
// word; the previous chunk's image imgo is cleared after B1.
//
// NQ = 0: the stores are inline asm, uncounted by the compiler (a loop of
// data-dependent length).  NQ > 0: exactly NQ 16-byte stores and one 4-byte
// store per thread, those with nothing to store past the buffer range
// (dropped), as compiler builtins: the compiler then counts them, and its
// wait for a prefetch issued before them lets them stay in flight (with NQ =
// 0 that wait, vmcnt(n) for the n loads it knows of, also waited for the
// uncounted stores, which are younger).  Quads past NQ per thread (chunks of
// long codes) go out uncounted, as with NQ = 0.
template <int ENC, bool RICE, uint32_t NT = CW_THREADS, uint32_t NQ = 0u>
__device__ __forceinline__ void cw_chunk(CwState &st, uint32_t *img, uint32_t *imgo, uint32_t (*s_wsum)[NT / 64u],
					 uint32_t par, uint32_t T, const uint32_t (&mp)[EPT / 2],
					 const uint32_t (&oq)[EPT / 2], const Coder &cd, bool fast, const char *tab,
					 u32x4 dst_rsrc)
{
	const uint32_t tid = threadIdx.x, lane = tid & 63u;
	const uint32_t wid = __builtin_amdgcn_readfirstlane(tid >> 6);
	const uint32_t inc = wave_incl_scan(T);
	if (lane == 63u)
		s_wsum[par][wid] = inc;
	lds_barrier(); // B1: wave totals
	for (uint32_t i = tid; i < st.used_prev; i += NT)
		imgo[i] = 0u;
	const uint32_t ws = lane < (NT / 64u) ? s_wsum[par][lane] : 0u;
	const uint32_t wsc = wave_incl_scan(ws);
	const uint32_t A = (uint32_t)__builtin_amdgcn_readlane((int)wsc, (NT / 64u) - 1);
	const uint32_t wex = wid ? (uint32_t)__builtin_amdgcn_readlane((int)wsc, (int)wid - 1) : 0u;
	const uint32_t r = st.P & 31u;
	walk_pack<ENC, RICE>(img, r + wex + inc - T, mp, oq, cd, fast, tab);
	if (tid == 0u && r)
		__hip_atomic_fetch_or(reinterpret_cast<lds_u32 *>((uintptr_t)img), st.carry, __ATOMIC_RELAXED,
				      __HIP_MEMORY_SCOPE_WORKGROUP);
	lds_barrier(); // B2: the packed image
	const uint32_t end = r + A, nfull = end >> 5;
	const lds_u32 *Ll = reinterpret_cast<const lds_u32 *>((uintptr_t)img);
	const uint32_t g0 = st.P >> 5;
	if constexpr (NQ == 0u) {
		for (uint32_t p = tid; p < (nfull >> 2); p += NT) {
			const u32x4 wv = *reinterpret_cast<const __attribute__((address_space(3))) u32x4 *>(Ll + 4u * p);
			u32x4 o;
			o.x = bswap32(wv.x);
			o.y = bswap32(wv.y);
			o.z = bswap32(wv.z);
			o.w = bswap32(wv.w);
			store_b128_nc(o, 4u * (g0 + 4u * p), dst_rsrc);
		}
		const uint32_t rr = (tid - (nfull >> 2)) & (NT - 1u);
		if (rr < (nfull & 3u)) {
			const uint32_t jw = (nfull & ~3u) + rr;
			store_b32_nc(bswap32(Ll[jw]), 4u * (g0 + jw), dst_rsrc);
		}
	} else {
		__amdgpu_buffer_rsrc_t rs;
		__builtin_memcpy(&rs, &dst_rsrc, sizeof(rs));
		const uint32_t nquad = nfull >> 2;
#pragma unroll
		for (uint32_t i = 0; i < NQ; i++) {
			const uint32_t p = tid + i * NT;
			const bool in = p < nquad;
			const u32x4 wv = *reinterpret_cast<const __attribute__((address_space(3))) u32x4 *>(Ll + (in ? 4u * p : 0u));
			u32x4 o;
			o.x = bswap32(wv.x);
			o.y = bswap32(wv.y);
			o.z = bswap32(wv.z);
			o.w = bswap32(wv.w);
			__builtin_amdgcn_raw_buffer_store_b128(o, rs, in ? (int)(4u * (g0 + 4u * p)) : INT32_MIN, 0, 0);
		}
		const uint32_t rr = (tid - nquad) & (NT - 1u);
		const bool part = rr < (nfull & 3u);
		const uint32_t jw = part ? (nfull & ~3u) + rr : 0u;
		__builtin_amdgcn_raw_buffer_store_b32(bswap32(Ll[jw]), rs, part ? (int)(4u * (g0 + jw)) : INT32_MIN, 0, 0);
		// a chunk longer than NQ quads per thread (long codes): the rest
		// uncounted, as with NQ = 0
		for (uint32_t p = tid + NQ * NT; p < nquad; p += NT) {
			const u32x4 wv = *reinterpret_cast<const __attribute__((address_space(3))) u32x4 *>(Ll + 4u * p);
			u32x4 o;
			o.x = bswap32(wv.x);
			o.y = bswap32(wv.y);
			o.z = bswap32(wv.z);
			o.w = bswap32(wv.w);
			store_b128_nc(o, 4u * (g0 + 4u * p), dst_rsrc);
		}
	}
	st.carry = (end & 31u) ? __builtin_amdgcn_readfirstlane(Ll[nfull]) : 0u;
	st.used_prev = nfull + 1u;
	st.P += A;
}

// Frame epilogue (cmp.c:314-334), one thread: zero-padded final bytes
// (bitstream_flush), checksum, header dwords, status (and needed)
__device__ __forceinline__ void cw_epilogue(uint8_t *fdst, uint32_t cap, uint32_t endbit, uint32_t carry, uint32_t HB,
					    bool checksum, uint32_t ck, const uint32_t (&h4)[5], uint32_t *status,
					    uint32_t *needed, uint32_t frame, uint32_t size)
{
	if (endbit & 31u) {
		const uint32_t nbytes = ((endbit & 31u) + 7u) >> 3;
		for (uint32_t b = 0; b < nbytes; b++)
			if (4u * (endbit >> 5) + b < cap)
				fdst[4u * (endbit >> 5) + b] = (uint8_t)(carry >> (24u - 8u * b));
	}
	const uint32_t payload_bytes = (endbit + 7u) >> 3;
	if (checksum)
		for (uint32_t b = 0; b < 4u; b++)
			if (payload_bytes + b < cap)
				fdst[payload_bytes + b] = (uint8_t)(ck >> (24u - 8u * b));
	const uint32_t hwords = HB == 176u ? 5u : 4u;
	for (uint32_t wq = 0; wq < hwords; wq++)
		if (4u * wq + 4u <= cap)
			*reinterpret_cast<uint32_t *>(fdst + 4u * wq) = bswap32(h4[wq]);
	status[frame] = size > cap ? ERRV(E_DST_TOO_SMALL) : size > 0xFFFFFFu ? ERRV(E_HDR_CMP_SIZE_TOO_LARGE) : size;
	if (needed)
		needed[frame] = size;
}

// The uncompressed fallback of frame f inside the context walk (cmp.c:342-393,
// after cmp_reset: NONE + UNCOMPRESSED, compress_engine with sequence number
// 0): the 16-byte header, the samples as big-endian 16-bit words (the low
// halves for i16-in-i32, sample_reader.h), the checksum, status = raw size;
// the model takes the samples (a primary pass, cmp.c:305-306).  The samples
// are read again (the walk keeps only the model).  The attempt's stores are
// uncounted asm stores: every wave drains them before the barrier, so the raw
// bytes land after them.
template <int W, int CH>
__device__ __forceinline__ void cw_fallback(const WArgs &a, uint32_t f, uint8_t *fdst, uint64_t id, uint32_t flip,
					 uint32_t (&mdl)[CH][EPT / 2])
{
	constexpr uint32_t RW = EPT * W / 16u;
	const uint32_t tid = threadIdx.x;
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__syncthreads();
	const u32x4 rsrc = rsrc_words(fdst, a.raw_size & ~3u);
	const uint8_t *fs = a.src + (uint64_t)f * a.src_stride;
#pragma unroll
	for (uint32_t cc = 0; cc < CH; cc++) {
		const uint32_t first = cc * CW_CHUNK + tid * EPT;
		const uint4 *p = reinterpret_cast<const uint4 *>(fs + (size_t)first * W);
		uint4 r[RW];
#pragma unroll
		for (uint32_t q = 0; q < RW; q++)
			r[q] = p[q];
		uint32_t w[EPT / 2];
		cw_pairs<W>(r, flip, w);
#pragma unroll
		for (uint32_t q = 0; q < EPT / 2; q++) {
			mdl[cc][q] = w[q];
			const uint32_t x = w[q] ^ flip; // the samples
			w[q] = ((x & 0x00FF00FFu) << 8) | ((x >> 8) & 0x00FF00FFu);
		}
#pragma unroll
		for (uint32_t q = 0; q < EPT / 8; q++)
			store_b128_nc((u32x4){w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]}, 16u + 2u * first + 16u * q,
				      rsrc);
	}
	if (tid == 0u) {
		uint32_t h[5];
		header_words(h, a.raw_size, 2u * a.n, id, 0u, PRE_NONE, a.checksum ? 1u : 0u, ENC_RAW, 0u, 0u, 0u);
#pragma unroll
		for (uint32_t wq = 0; wq < 4u; wq++)
			store_b32_nc(bswap32(h[wq]), 4u * wq, rsrc);
		if (a.checksum)
			store_b32_nc(bswap32(a.checksums[f]), 16u + 2u * a.n, rsrc);
		a.status[f] = a.raw_size;
	}
}

template <int W, int PRE_P, int ENC_P, bool RICE_P, int ENC_S, bool RICE_S, int CH>
__global__ __launch_bounds__(1024) void walk_ctx_kernel(WArgs a)
{
	static_assert(CH % 2 == 0, "two images alternate within a frame");
	constexpr uint32_t RW = EPT * W / 16u; // uint4 per lane
	extern __shared__ __attribute__((aligned(16))) uint32_t L_img[];
	__shared__ uint32_t s_wsum[2][CW_WAVES];
	__shared__ __attribute__((aligned(16))) uint2 s_tab[2][WTAB];

	const uint32_t tid = threadIdx.x, lane = tid & 63u;
	const uint32_t c = blockIdx.x;
	const uint32_t n = a.n; // CH * CW_CHUNK
	uint16_t *mbase = reinterpret_cast<uint16_t *>(a.model_ptrs ? (uint8_t *)(uintptr_t)a.model_ptrs[c]
								    : a.model + (uint64_t)c * a.model_stride);
	// two images of img_words words, each after a 4-word pad (the packer's
	// first put may OR the word before its image)
	uint32_t *const img0 = L_img + 4, *const img1 = L_img + 4 + a.img_words;

	const Coder cp = make_coder<ENC_P>(a.g_p, a.outl_p);
	const Coder cs = make_coder<ENC_S>(a.g_s, a.outl_s);
	const bool fast_p = RICE_P && (ENC_P == ENC_MULTI || (ENC_P == ENC_ZERO && cp.k <= 11u));
	const bool fast_s = RICE_S && (ENC_S == ENC_MULTI || (ENC_S == ENC_ZERO && cs.k <= 11u));
	if (tid < WTAB) {
		if (fast_p)
			s_tab[0][tid] = walk_table_entry<ENC_P>(tid, cp);
		if (fast_s)
			s_tab[1][tid] = walk_table_entry<ENC_S>(tid, cs);
	}
	for (uint32_t i = tid; i < 2u * a.img_words + 4u; i += CW_THREADS)
		L_img[i] = 0u;

	const uint32_t seq0 = a.seq0s ? a.seq0s[c] : a.seq0;
	const uint32_t flip = a.is_unsigned ? 0u : 0x80008000u; // see walk_kernel
	uint32_t mdl[CH][EPT / 2];
#pragma unroll
	for (uint32_t cc = 0; cc < CH; cc++)
#pragma unroll
		for (uint32_t q = 0; q < EPT / 2; q++)
			mdl[cc][q] = 0u;
	if (seq0 != 0u && seq0 <= a.iters) { // the first frame is a secondary pass
#pragma unroll
		for (uint32_t cc = 0; cc < CH; cc++) {
			const uint4 *mp4 = reinterpret_cast<const uint4 *>(mbase + cc * CW_CHUNK + tid * EPT);
#pragma unroll
			for (uint32_t q = 0; q < EPT / 8; q++) {
				const uint4 v = mp4[q];
				mdl[cc][4 * q] = v.x ^ flip;
				mdl[cc][4 * q + 1] = v.y ^ flip;
				mdl[cc][4 * q + 2] = v.z ^ flip;
				mdl[cc][4 * q + 3] = v.w ^ flip;
			}
		}
	}
	// samples of step s (= acquisition s / CH, chunk s % CH): register set
	// s % CW_DEPTH
	const uint32_t steps = a.fpc * CH;
	uint4 rs[CW_DEPTH][RW];
	uint32_t pv[CW_DEPTH];
#pragma unroll
	for (uint32_t d = 0; d < CW_DEPTH; d++)
		pv[d] = 0u;
	// unconditional loads (a step past the end reloads the last chunk): a
	// conditional load into live registers makes the compiler wait for it
	auto issue = [&](uint32_t set, uint32_t step) {
		step = step < steps ? step : steps - 1u;
		const uint32_t acq = step / CH, cc = step % CH;
		const uint8_t *fs = a.src + (uint64_t)(c * a.fpc + acq) * a.src_stride;
		const uint32_t first = cc * CW_CHUNK + tid * EPT;
		const uint4 *p = reinterpret_cast<const uint4 *>(fs + (size_t)first * W);
#pragma unroll
		for (uint32_t q = 0; q < RW; q++)
			rs[set][q] = p[q];
		if (PRE_P == PRE_DIFF) {
			const uint32_t ip = first ? first - 1u : 0u;
			pv[set] = W == 2 ? (uint32_t)reinterpret_cast<const uint16_t *>(fs)[ip]
					 : reinterpret_cast<const uint32_t *>(fs)[ip];
		}
	};
#pragma unroll
	for (uint32_t d = 0; d < CW_DEPTH; d++)
		if (d < steps)
			issue(d, d);
	__syncthreads(); // tables and the zeroed images

	const char *tab_p = reinterpret_cast<const char *>(s_tab[0]);
	const char *tab_s = reinterpret_cast<const char *>(s_tab[1]);
	uint32_t sq = seq0;
	CwState st;
	st.used_prev = 0u;
	// Frame epilogues (header words, final bytes, checksum, status: partial
	// cache lines) of up to AIRS_WALK_EPI_MAX frames are kept in LDS, four
	// words per frame, and written after the walk (as the segment walk's,
	// DESIGN.md 3.7): in the loop, the next waits of wave 0 covered them
	const bool defer = a.fpc <= AIRS_WALK_EPI_MAX;
	uint32_t *const epi = L_img + 4u + 2u * a.img_words;
	if (defer && tid < a.fpc)
		epi[4u * tid + 3u] = 0u; // no epilogue (a fallback frame) until written
	auto frame_id = [&](uint32_t ai) {
		return a.ids ? a.ids[c * a.fpc + ai] : a.id_base + (uint64_t)c * a.id_cstep + (uint64_t)ai * a.id_astep;
	};
	// frame ai: total size, end bit, carry word, meta = header sequence number
	// | primary << 8 | 22-byte header << 9
	auto frame_epilogue = [&](uint32_t ai, uint32_t size, uint32_t endbit, uint32_t carry, uint32_t meta) {
		const uint32_t fr = c * a.fpc + ai;
		const uint64_t id = frame_id(ai);
		uint32_t h[5];
		if (meta & 0x100u)
			header_words(h, size, 2u * n, id, meta & 0xFFu, PRE_P, a.checksum ? 1u : 0u, ENC_P, 0u,
				     ENC_P == ENC_RAW ? 0u : cp.g, ENC_P == ENC_RAW ? 0u : cp.outlier);
		else
			header_words(h, size, 2u * n, id, meta & 0xFFu, PRE_MODEL, a.checksum ? 1u : 0u, ENC_S, a.model_rate,
				     ENC_S == ENC_RAW ? 0u : cs.g, ENC_S == ENC_RAW ? 0u : cs.outlier);
		cw_epilogue(a.dst + (uint64_t)fr * a.dst_stride, a.cap, endbit, carry, (meta & 0x200u) ? 176u : 128u,
			    a.checksum != 0u, a.checksum ? a.checksums[fr] : 0u, h, a.status, nullptr, fr, size);
	};
	for (uint32_t acq = 0; acq < a.fpc; acq++) {
		const uint32_t f = c * a.fpc + acq;
		const bool prim = sq == 0u || sq > a.iters; // cmp.c:228-248
		const uint32_t hseq = prim ? 0u : sq;
		sq = prim ? 1u : sq + 1u;
		const uint32_t HB = prim ? hdr_bits(PRE_P, ENC_P) : hdr_bits(PRE_MODEL, ENC_S);
		const uint32_t enc = prim ? (uint32_t)ENC_P : (uint32_t)ENC_S;
		// the frame's first payload word starts with header bytes 20-21
		st.P = HB;
		st.carry = (HB & 31u) && enc != ENC_RAW ? ((prim ? cp.outlier : cs.outlier) & 0xFFFFu) << 16 : 0u;
		uint8_t *fdst = a.dst + (uint64_t)f * a.dst_stride;
		const u32x4 dst_rsrc = rsrc_words(fdst, a.cap & ~3u);
#pragma unroll
		for (uint32_t cc = 0; cc < CH; cc++) {
			const uint32_t step = acq * CH + cc;
			uint32_t w[EPT / 2];
			cw_pairs<W>(rs[cc % CW_DEPTH], flip, w);
			const uint32_t prevs = (cc != 0u || tid >= 64u) ? pv[cc % CW_DEPTH] & 0xFFFFu : 0u;
			issue(cc % CW_DEPTH, step + CW_DEPTH); // lands while the chunks before it are coded
			uint32_t mp[EPT / 2], oq[EPT / 2];
			uint32_t T;
			if (prim) {
				cw_primary<PRE_P, ENC_P>(w, prevs, flip, lane, mp);
#pragma unroll
				for (uint32_t q = 0; q < EPT / 2; q++)
					mdl[cc][q] = w[q]; // cmp.c:305-306
				T = walk_lengths<ENC_P, RICE_P>(mp, oq, cp, fast_p, tab_p);
			} else {
				const int32_t r1 = 16 - (int32_t)a.model_rate;
#pragma unroll
				for (uint32_t q = 0; q < EPT / 2; q++) {
					const uint32_t u = unpk(pk(w[q]) - pk(mdl[cc][q])); // preprocess.c:406-411
					mp[q] = ENC_S == ENC_RAW ? u : zigzag_pk(u);
					mdl[cc][q] = model_update_zx(w[q], mdl[cc][q], r1); // cmp.c:132-142
				}
				T = walk_lengths<ENC_S, RICE_S>(mp, oq, cs, fast_s, tab_s);
			}
#pragma unroll
			for (uint32_t q = 0; q < EPT / 2; q++)
				asm volatile("" : "+v"(mp[q]), "+v"(oq[q]));
			uint32_t *const img = (cc & 1u) ? img1 : img0;
			uint32_t *const imgo = (cc & 1u) ? img0 : img1;
			if (prim)
				cw_chunk<ENC_P, RICE_P, CW_THREADS, CW_NQ>(st, img, imgo, s_wsum, cc & 1u, T, mp, oq, cp, fast_p,
									    tab_p, dst_rsrc);
			else
				cw_chunk<ENC_S, RICE_S, CW_THREADS, CW_NQ>(st, img, imgo, s_wsum, cc & 1u, T, mp, oq, cs, fast_s,
									    tab_s, dst_rsrc);
		}
		const uint32_t size = ((st.P + 7u) >> 3) + (a.checksum ? 4u : 0u);
		// the uncompressed fallback (cmp.c:342-393): the attempt ran with the
		// raw frame size as its capacity (a.cap); a frame that does not fit is
		// reset and written raw (block-uniform: st.P is)
		const bool fbk = a.fb && size > a.raw_size;
		// identifier draws: one per reset (cmp.c:228-231, 371-392); with the
		// deferred epilogues kept in the frame's record (bits 12-13)
		const uint32_t draws = prim ? (fbk ? 3u : 1u) : (fbk ? 2u : 0u);
		if (a.draws && tid == 0u && !defer)
			a.draws[f] = (uint8_t)draws;
		if (fbk) {
			if (defer && tid == 0u)
				epi[4u * acq + 3u] = draws << 12;
			cw_fallback<W, CH>(a, f, fdst, frame_id(acq), flip, mdl);
			sq = 1u; // the fallback frame has sequence number 0, the next 1
		} else if (tid == 0u) {
			const uint32_t meta = hseq | (prim ? 0x100u : 0u) | (HB == 176u ? 0x200u : 0u);
			if (defer) { // written after the walk (see frame_epilogue)
				uint32_t *const rec = epi + 4u * acq;
				rec[0] = size;
				rec[1] = st.P;
				rec[2] = st.carry;
				rec[3] = meta | 0x400u | draws << 12;
			} else {
				frame_epilogue(acq, size, st.P, st.carry, meta);
			}
		}
	}
	if (defer && tid < 64u) {
		// the epilogues kept in LDS (written by thread 0 in the loop; frames
		// that took the fallback have none)
		for (uint32_t ai = tid; ai < a.fpc; ai += 64u) {
			const uint32_t *const rec = epi + 4u * ai;
			if (a.draws)
				a.draws[c * a.fpc + ai] = (uint8_t)((rec[3] >> 12) & 3u);
			if (rec[3] & 0x400u)
				frame_epilogue(ai, rec[0], rec[1], rec[2], rec[3]);
		}
	}
	if (a.seq_out && tid == 0u)
		a.seq_out[c] = (uint8_t)sq;
	// the model after the last acquisition, to the work buffer (cmp.c:304-311)
#pragma unroll
	for (uint32_t cc = 0; cc < CH; cc++) {
		uint4 *mo = reinterpret_cast<uint4 *>(mbase + cc * CW_CHUNK + tid * EPT);
#pragma unroll
		for (uint32_t q = 0; q < EPT / 8; q++)
			mo[q] = make_uint4(mdl[cc][4 * q] ^ flip, mdl[cc][4 * q + 1] ^ flip, mdl[cc][4 * q + 2] ^ flip,
					   mdl[cc][4 * q + 3] ^ flip);
	}
}

// ---------------------------------------------------------------------
// launch (airs_dev_walk, airs_dev.h)
// ---------------------------------------------------------------------
// the segment walk's launch: the block index is the logical index when the
// whole grid is resident at once (occupancy of this kernel x CUs), else a ticket
//
// Direct launches assume that every workgroup of the grid is running, so a
// look-back only ever waits on a running workgroup.  That holds only when
// nothing else occupies the device: the engine must be marked exclusive
// (CMP_GPU_OPT_EXCLUSIVE), and the grid must fit what the CUs admit.  The
// occupancy API reads one block per CU high at some SGPR counts
// (MI355X_MICROARCH.md "Residency"), so the count is also capped by the
// guide's SGPR rule at the largest allocation a kernel can have (102 SGPRs +
// VCC: 112 per wave, 800 per SIMD: 6 waves per SIMD).  Otherwise each
// workgroup takes its logical index from the ticket counter as it starts.
template <typename K>
static int walk_go(K kern, const WArgs &k, size_t lds, hipStream_t s, bool exclusive)
{
	const uint32_t grid = k.num_ctx * k.spf;
	int dev = 0, cus = 0, per_cu = 0;
	if (hipGetDevice(&dev) != hipSuccess ||
	    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
		cus = 0;
	if (cus > 0 && hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 320, lds) != hipSuccess)
		per_cu = 0;
	WArgs kk = k;
	const int sgpr_cap = 4 * (800 / (112 + 16)) / 5; // 320-thread (5-wave) blocks per CU
	per_cu = per_cu < sgpr_cap ? per_cu : sgpr_cap;
	kk.direct =
		(exclusive && cus > 0 && per_cu > 0 && (uint64_t)grid <= (uint64_t)per_cu * (uint64_t)cus) ? 1u : 0u;
	kk.cus = cus > 0 ? (uint32_t)cus : 0u;
	hipLaunchKernelGGL(kern, dim3(grid), dim3(320), lds, s, kk);
	return kk.direct ? 1 : 0;
}

// < 0: no kernel for these passes; 0: launched with the ticket; 1: direct
template <int W, int PRE_P, int ENC_P, bool RICE_P>
static int walk_launch_s(const WArgs &k, uint32_t enc_s, bool rice_s, size_t lds, hipStream_t s, bool ex)
{
	const bool half = k.spf * walk_seg_samples(true) == k.n && k.spf * walk_seg_samples(false) != k.n;
	if (enc_s == ENC_ZERO && rice_s)
		return half ? walk_go(walk_kernel<W, PRE_P, ENC_P, RICE_P, ENC_ZERO, true, 8>, k, lds, s, ex)
			    : walk_go(walk_kernel<W, PRE_P, ENC_P, RICE_P, ENC_ZERO, true, 16>, k, lds, s, ex);
	if (enc_s == ENC_MULTI && rice_s)
		return half ? walk_go(walk_kernel<W, PRE_P, ENC_P, RICE_P, ENC_MULTI, true, 8>, k, lds, s, ex)
			    : walk_go(walk_kernel<W, PRE_P, ENC_P, RICE_P, ENC_MULTI, true, 16>, k, lds, s, ex);
	return -1;
}

// samples per segment of the segment walk: 256 lanes of 16 samples, or of 8
uint32_t walk_seg_samples(bool half)
{
	return half ? 2048u : 4096u;
}

template <int W, int PRE_P>
static int walk_launch_p(const WArgs &k, uint32_t enc_p, bool rice_p, uint32_t enc_s, bool rice_s, size_t lds,
			 hipStream_t s, bool ex)
{
	if (enc_p == ENC_ZERO && rice_p)
		return walk_launch_s<W, PRE_P, ENC_ZERO, true>(k, enc_s, rice_s, lds, s, ex);
	if (enc_p == ENC_MULTI && rice_p)
		return walk_launch_s<W, PRE_P, ENC_MULTI, true>(k, enc_s, rice_s, lds, s, ex);
	return -1;
}

template <int W, int PRE_P, int ENC_P, bool RICE_P>
static bool walk_ctx_launch_s(const WArgs &k, uint32_t enc_s, bool rice_s, size_t lds, hipStream_t s)
{
	const dim3 grid(k.num_ctx), blk(CW_THREADS);
	if (enc_s == ENC_ZERO && rice_s)
		hipLaunchKernelGGL((walk_ctx_kernel<W, PRE_P, ENC_P, RICE_P, ENC_ZERO, true, 4>), grid, blk, lds, s, k);
	else if (enc_s == ENC_MULTI && rice_s)
		hipLaunchKernelGGL((walk_ctx_kernel<W, PRE_P, ENC_P, RICE_P, ENC_MULTI, true, 4>), grid, blk, lds, s, k);
	else
		return false;
	return true;
}

template <int W, int PRE_P>
static bool walk_ctx_launch_p(const WArgs &k, uint32_t enc_p, bool rice_p, uint32_t enc_s, bool rice_s, size_t lds,
			      hipStream_t s)
{
	if (enc_p == ENC_ZERO && rice_p)
		return walk_ctx_launch_s<W, PRE_P, ENC_ZERO, true>(k, enc_s, rice_s, lds, s);
	if (enc_p == ENC_MULTI && rice_p)
		return walk_ctx_launch_s<W, PRE_P, ENC_MULTI, true>(k, enc_s, rice_s, lds, s);
	return false;
}

// walk_ctx_kernel's two images, then the deferred frame epilogues
static size_t walk_ctx_lds_dyn(uint32_t img_words, uint32_t fpc)
{
	return (size_t)(2u * img_words + 4u) * 4u + (fpc <= AIRS_WALK_EPI_MAX ? (size_t)fpc * 16u : 0u);
}

// walk_kernel's images, then the deferred frame epilogues
static size_t walk_seg_lds_dyn(uint32_t img_words, uint32_t fpc)
{
	return (size_t)(AIRS_WALK_NIMG * (img_words + 4u) + 4u) * 4u + (fpc <= AIRS_WALK_EPI_MAX ? (size_t)fpc * 16u : 0u);
}

// the static arrays of the two kernels (tables, wave sums, a few words),
// bounded from above
#define WALK_STATIC_LDS (2u * WTAB * 8u + 2u * 16u * 4u + 256u)

size_t walk_ctx_lds(uint32_t img_words, uint32_t fpc)
{
	return walk_ctx_lds_dyn(img_words, fpc) + WALK_STATIC_LDS;
}

size_t walk_seg_lds(uint32_t img_words, uint32_t fpc)
{
	return walk_seg_lds_dyn(img_words, fpc) + WALK_STATIC_LDS;
}

uint32_t walk_ctx_samples()
{
	return 4u * CW_CHUNK;
}

bool walk_ctx_encode(const WArgs &k, uint32_t sample_bytes, uint32_t pre_p, uint32_t enc_p, bool rice_p,
		     uint32_t enc_s, bool rice_s, hipStream_t s)
{
	if (k.n != 4u * CW_CHUNK)
		return false;
	const size_t lds = walk_ctx_lds_dyn(k.img_words, k.fpc);
	if (walk_ctx_lds(k.img_words, k.fpc) > AIRS_LDS_BYTES)
		return false;
	if (sample_bytes == 2)
		return pre_p == PRE_DIFF ? walk_ctx_launch_p<2, PRE_DIFF>(k, enc_p, rice_p, enc_s, rice_s, lds, s)
					 : walk_ctx_launch_p<2, PRE_NONE>(k, enc_p, rice_p, enc_s, rice_s, lds, s);
	return pre_p == PRE_DIFF ? walk_ctx_launch_p<4, PRE_DIFF>(k, enc_p, rice_p, enc_s, rice_s, lds, s)
				 : walk_ctx_launch_p<4, PRE_NONE>(k, enc_p, rice_p, enc_s, rice_s, lds, s);
}

int walk_encode(const WArgs &k, uint32_t sample_bytes, uint32_t pre_p, uint32_t enc_p, bool rice_p, uint32_t enc_s,
		bool rice_s, hipStream_t s, bool exclusive)
{
	const size_t lds = walk_seg_lds_dyn(k.img_words, k.fpc);
	if (walk_seg_lds(k.img_words, k.fpc) > AIRS_LDS_BYTES)
		return -1;
	if (sample_bytes == 2)
		return pre_p == PRE_DIFF ? walk_launch_p<2, PRE_DIFF>(k, enc_p, rice_p, enc_s, rice_s, lds, s, exclusive)
					 : walk_launch_p<2, PRE_NONE>(k, enc_p, rice_p, enc_s, rice_s, lds, s, exclusive);
	return pre_p == PRE_DIFF ? walk_launch_p<4, PRE_DIFF>(k, enc_p, rice_p, enc_s, rice_s, lds, s, exclusive)
				 : walk_launch_p<4, PRE_NONE>(k, enc_p, rice_p, enc_s, rice_s, lds, s, exclusive);
}

} // namespace airs
