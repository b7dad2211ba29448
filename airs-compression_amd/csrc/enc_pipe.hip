// enc_pipe.hip -- the persistent, software-pipelined encode kernel (gfx950).
//
// Same per-sample work as encode_kernel (reference cmp.c:296-312: predictor,
// ZigZag encoder.c:274-286, Golomb encoder.c:303-378, big-endian bit packing
// bitstream_writer.h:124-158) and the same decoupled look-back over 8-byte
// granules, but arranged so that no segment waits for a segment that is
// still loading its samples:
//
//   * the grid is the number of co-resident workgroups G; workgroup w
//     encodes the dispatch indices d = w, w + G, w + 2G, ... (frame-
//     interleaved: consecutive d are the same segment index of consecutive
//     frames, as in encode_kernel)
//   * iteration i packs segment d_i while phase 1 of d_{i+1} (residuals,
//     code lengths, the published aggregate and tail) runs in the same
//     iteration, and the samples of d_{i+2} stream into LDS meanwhile
//     (global_load_lds, issued one iteration ahead)
//   * so every aggregate a look-back needs was published an iteration
//     earlier: the look-back of d_i is one granule round trip, overlapped
//     with the packing of d_i, and a slow load holds up only its own
//     workgroup, never the chain of its frame.
//
// Wave roles.  The memory counter vmcnt is per wave and retires in order, so
// a wait for one access also waits for every older one.  Wave 0 owns the
// look-back (granule loads and stores) and the frame epilogue; waves 1-2
// store the images; wave 3 issues the LDS-DMA prefetch (and the tail
// granule).  So no wave ever waits for a slower kind of access than the one
// it needs.  Workgroup barriers are LDS-only
// (s_waitcnt lgkmcnt(0) + s_barrier) so the prefetch stays in flight across
// them (cdna_hip_programming.md, "Pipelining across barriers"); uniform
// per-frame values come through scalar loads.
//
// A segment is PCH chunks of 4096 samples (two for 16-bit input, one for
// 32-bit): lane t owns samples [16t, 16t+16) of each chunk.
//
// Deadlock freedom: a segment waits only for segments with a smaller
// dispatch index, and every workgroup of the grid is resident (the host
// sizes G from the occupancy query), so the smallest unfinished segment can
// always proceed.  Spins are bounded as in encode_kernel.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "enc_common.h"

namespace airs {

__host__ __device__ constexpr uint32_t pipe_chunks(int W)
{
	return W == 2 ? 2u : 1u;
}

// LDS-only workgroup barrier: outstanding global loads and LDS-DMA are not
// drained, unlike __syncthreads()'s fence
__device__ __forceinline__ void lds_barrier()
{
	asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// wave-uniform 32-bit load through the scalar cache (read-only data the host
// wrote before the launch); lgkmcnt, so it never waits on the vmcnt queue
__device__ __forceinline__ uint32_t sload32(const uint32_t *p)
{
	uint32_t v;
	asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
	return v;
}

__device__ __forceinline__ uint64_t sload64(const uint64_t *p)
{
	uint64_t v;
	asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
	return v;
}

// Loads the compiler does not see.  Every vector load of this kernel goes
// through these, with explicit waits: the compiler's own waitcnt insertion
// is conservative at control-flow merges (vmcnt(0) in code all waves run),
// which would drain waves 1-3's prefetch.  Ordering: the memory clobber
// keeps them in program order with the other memory accesses, and a value
// is only read after a wait that names it as an operand.
//
// LDS-DMA: 16 bytes per lane from g to LDS byte lds + 16 * lane (M0 base).
// M0 is saved and restored around it (it is reserved to the compiler).
__device__ __forceinline__ void dma16(const void *g, uint32_t lds)
{
	uint32_t keep;
	asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
		     "s_mov_b32 m0, %0"
		     : "=&s"(keep)
		     : "v"(g), "s"(lds)
		     : "memory");
}

// granule load (agent scope, as gran_load), no wait
__device__ __forceinline__ uint64_t gran_issue(const uint64_t *p)
{
	uint64_t v;
	asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
	return v;
}

// granule load and wait
__device__ __forceinline__ uint64_t gran_fetch(const uint64_t *p)
{
	uint64_t v;
	asm volatile("global_load_dwordx2 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
	return v;
}

__device__ __forceinline__ void vm_wait2(uint64_t &x, uint64_t &y)
{
	asm volatile("s_waitcnt vmcnt(0)" : "+v"(x), "+v"(y)::"memory");
}

__device__ __forceinline__ void vm_wait()
{
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Timeline stamps (-DAIRS_PIPE_TS=1 builds with AIRS_DBG=65536): per segment
// being packed, 8 slots of the 100 MHz realtime clock: 0 iteration start,
// 1 packed, 2 phase 1 of the next segment done, 3 look-back done, 4 stored,
// 5 images cleared, 7 workgroup | XCC << 32
#ifndef AIRS_PIPE_TS
#define AIRS_PIPE_TS 0
#endif
__device__ __forceinline__ void pipe_stamp(const KArgs &a, uint32_t gseg, uint32_t slot, uint32_t tid)
{
	if (AIRS_PIPE_TS && a.dbgts && tid == 0) {
		uint64_t t;
		asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t));
		a.dbgts[8u * gseg + slot] = t;
		if (slot == 0) {
			uint32_t xcc;
			asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
			a.dbgts[8u * gseg + 7u] = ((uint64_t)xcc << 32) | blockIdx.x;
		}
	}
}

// experiment switches: AIRS_PIPE_PF 1 issues the prefetch during the image
// stores instead of right after phase 1; AIRS_PIPE_PRIO 1 raises the issue
// priority of younger workgroups (dispatch slot on the CU), so the four
// workgroups of a CU advance at the same pace
#ifndef AIRS_PIPE_PF
#define AIRS_PIPE_PF 0
#endif
#ifndef AIRS_PIPE_PRIO
#define AIRS_PIPE_PRIO 0
#endif

// wave-uniform state of one segment
template <uint32_t NC>
struct PSeg {
	uint32_t d, frame, lf, gseg, sif, first_seg;
	uint32_t A;        // bits of the segment
	uint32_t tot[NC];  // bits per chunk
	uint32_t gpar;     // Golomb parameter of the frame
	uint32_t fastk;    // Rice/ZERO table path
	Coder cd;
};

template <uint32_t NC>
__device__ __forceinline__ void pseg_locate(const KArgs &a, uint32_t d, uint32_t nfr, PSeg<NC> &s)
{
	s.d = d;
	s.sif = d / nfr;
	s.lf = d - s.sif * nfr;
	s.gseg = s.lf * a.segs_per_frame + s.sif;
	s.first_seg = s.gseg - s.sif;
	s.frame = a.frame_list ? sload32(a.frame_list + s.lf) : a.frame_add + s.lf * a.frame_mul;
}

// LDS staging of one segment: DMA instruction ii = (c*4 + wave)*RW + q moves
// the 16-byte piece q of every lane of that wave's part of chunk c, lane l to
// byte 16 l of slot ii (1 KiB).  After the NI slots: the 16 bytes before the
// segment (DIFF needs the sample before it).
template <int W>
struct Stage {
	static constexpr uint32_t NC = pipe_chunks(W);
	static constexpr uint32_t RW = EPT * W / 16u;  // 16-byte pieces per lane per chunk
	static constexpr uint32_t NI = NC * 4u * RW;   // DMA instructions per segment (16)
	static constexpr uint32_t BYTES = NI * 1024u + 16u;
};

// Issue the LDS-DMA of segment (frame, sif) into the staging area (wave 3
// only; no wait).
template <int W, int PRE>
__device__ __forceinline__ void pipe_prefetch(const KArgs &a, uint32_t frame, uint32_t sif, uint32_t lane,
					      uint32_t *stage)
{
	using S = Stage<W>;
	const uint8_t *fsrc = a.src + (uint64_t)frame * a.src_stride;
	const uint8_t *seg = fsrc + (size_t)sif * (S::NC * AIRS_SEG) * W;
	const uint32_t sb = (uint32_t)(uintptr_t)stage; // LDS byte address
#pragma unroll
	for (uint32_t ii = 0; ii < S::NI; ii++) {
		const uint32_t q = ii % S::RW, wv = (ii / S::RW) % 4u, c = ii / (S::RW * 4u);
		const uint8_t *g = seg + ((size_t)c * AIRS_SEG + (64u * wv + lane) * EPT) * W + 16u * q;
		dma16(g, __builtin_amdgcn_readfirstlane(sb + ii * 1024u));
	}
	if (PRE == PRE_DIFF && sif != 0u && lane == 0u)
		dma16(seg - 16, __builtin_amdgcn_readfirstlane(sb + S::NI * 1024u));
}

// Look-back (wave 0): exclusive bit offset of segment gseg inside its frame
// stream (header bits included), from the aggregates of the segments before
// it back to the nearest inclusive prefix.  gv = the first window, loaded
// earlier.  Every needed granule carries the launch epoch or is re-polled.
__device__ __forceinline__ uint32_t pipe_lookback(const KArgs &a, uint32_t gseg, uint32_t first_seg, uint32_t lane,
						  uint64_t gv, uint32_t &polls)
{
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
			// a needed predecessor has not published yet: poll this window again
			if (++spins > AIRS_SPIN_LIMIT) {
				if (lane == 0)
					atomicAdd(a.ticket + AIRS_FAULT_WORD, 1u);
				return sum;
			}
			polls++;
			__builtin_amdgcn_s_sleep(1);
		} else {
			sum += wave_sum((inr && lane <= fi) ? (uint32_t)gv : 0u);
			if (incl_m)
				return sum;
			j -= 64;
		}
		const int64_t nidx = j - (int64_t)lane;
		gv = gran_fetch(&a.agg[nidx >= (int64_t)first_seg ? nidx : (int64_t)first_seg]);
	}
}

template <int W, int PRE, int ENC, bool RICE>
__global__ __launch_bounds__(EWG) void encode_pipe_kernel(KArgs a, uint32_t G)
{
	using S = Stage<W>;
	constexpr uint32_t NC = S::NC;
	constexpr uint32_t RW = S::RW;
	constexpr uint32_t NPIECE = ENC == ENC_MULTI ? 2 : 1;
	constexpr bool EXT_HDR = !(PRE == PRE_NONE && ENC == ENC_RAW);
	constexpr uint32_t HDR_BITS = EXT_HDR ? 176u : 128u;
	static_assert(EWG == 256 && EPT == 16, "lane layout");

	// dynamic LDS: the staging area, then NC chunk images of a.img_words
	// words, each after a 4-word guard
	extern __shared__ __attribute__((aligned(16))) uint32_t L_dyn[];
	uint32_t *const stage = L_dyn;
	uint32_t *const imgs = L_dyn + S::BYTES / 4u;
	const uint32_t IMGW = a.img_words + 4u;
	__shared__ uint32_t s_wsum[NC][EWG / 64];
	__shared__ uint32_t s_misc[4];
	// Rice/ZERO code tables of the segment being packed and the one in
	// phase 1 (frames may differ in g): entry q' = min(q, 17) = {T'[q'], len}
	__shared__ __attribute__((aligned(16))) uint2 s_rice[2][20];

	const uint32_t tid = threadIdx.x, lane = tid & 63u;
	const uint32_t wid = __builtin_amdgcn_readfirstlane(tid >> 6);
	const uint32_t nfr = a.num_segs / a.segs_per_frame;

	uint32_t mp[NC][EPT / 2], mq[NC][EPT / 2]; // mapped values, table offsets 8 min(q, 17)
	uint32_t excl[NC];                          // lane's bit offset inside each chunk
	PSeg<NC> cur, nxt;
	uint32_t par = 0u; // s_rice slot of `cur`

	// zero the chunk images once; afterwards each is cleared after its store
	{
		uint4 *L4 = reinterpret_cast<uint4 *>(imgs);
		for (uint32_t i = tid; i < NC * IMGW / 4u; i += EWG)
			L4[i] = make_uint4(0u, 0u, 0u, 0u);
	}

	// ---- phase 1 of segment s from the staging area (residuals, lengths,
	// the aggregate and tail granules); its barrier is the last read of the
	// staging area, which may be refilled after it
	auto phase1 = [&](PSeg<NC> &s, uint32_t slot, bool pf, uint32_t pf_frame, uint32_t pf_sif) {
		s.gpar = a.frame_g ? sload32(a.frame_g + s.frame) : a.g;
		s.cd = make_coder<ENC>(ENC == ENC_RAW ? 1u : s.gpar, a.outlier_param);
		s.fastk = (ENC == ENC_ZERO && RICE && s.cd.k <= 11u) ? 1u : 0u;
		const bool fastk = s.fastk != 0u;
		if (fastk && tid < 18u)
			s_rice[slot][tid] = rice_table_entry(tid, s.cd.k);
		uint32_t T[NC];
#pragma unroll
		for (uint32_t c = 0; c < NC; c++) {
			uint4 raw[RW];
#pragma unroll
			for (uint32_t q = 0; q < RW; q++)
				raw[q] = *reinterpret_cast<const uint4 *>(stage + ((c * 4u + wid) * RW + q) * 256u + lane * 4u);
			uint32_t w[EPT / 2];
			if (W == 2) {
#pragma unroll
				for (uint32_t q = 0; q < RW; q++) {
					w[4 * q] = raw[q].x;
					w[4 * q + 1] = raw[q].y;
					w[4 * q + 2] = raw[q].z;
					w[4 * q + 3] = raw[q].w;
				}
			} else {
#pragma unroll
				for (uint32_t q = 0; q < RW; q++) {
					w[2 * q] = __builtin_amdgcn_perm(raw[q].y, raw[q].x, 0x05040100u);
					w[2 * q + 1] = __builtin_amdgcn_perm(raw[q].w, raw[q].z, 0x05040100u);
				}
			}
			uint32_t wprev = 0u;
			if (PRE == PRE_DIFF) {
				wprev = __shfl_up(w[EPT / 2 - 1], 1, 64);
				if (lane == 0u) {
					// the sample before the wave's first: the previous wave's (or
					// chunk's) last, or for the segment's first the staged 16
					// bytes before it; zero for the frame's first (r[0] = x[0])
					uint32_t pv;
					if (c == 0u && wid == 0u) {
						pv = stage[S::NI * 256u + 3u];
						pv = s.sif == 0u ? 0u : (W == 2 ? pv >> 16 : pv);
					} else {
						const uint32_t pw = wid ? (c * 4u + wid - 1u) : ((c - 1u) * 4u + 3u);
						pv = stage[(pw * RW + RW - 1u) * 256u + 63u * 4u + 3u];
						pv = W == 2 ? pv >> 16 : pv;
					}
					wprev = pv << 16;
				}
			}
#pragma unroll
			for (uint32_t j = 0; j < EPT / 2; j++) {
				uint32_t u = w[j];
				if (PRE == PRE_DIFF)
					u = unpk(pk(w[j]) - pk(__builtin_amdgcn_alignbit(w[j], j ? w[j - 1] : wprev, 16)));
				mp[c][j] = ENC == ENC_RAW ? u : zigzag_pk(u);
			}
			uint32_t t = 0u;
			if (fastk) {
				u16x2 acc = (u16x2)(0);
#pragma unroll
				for (uint32_t j = 0; j < EPT / 2; j++) {
					const u16x2 v = __builtin_elementwise_add_sat(pk(mp[c][j]), (u16x2)(1));
					const u16x2 q = v >> (u16x2)((unsigned short)s.cd.k);
					acc += __builtin_elementwise_min(q, (u16x2)(16));
					mq[c][j] = unpk(__builtin_elementwise_min(q, (u16x2)(17)) << (u16x2)(3));
				}
				t = EPT * (s.cd.k + 1u) + (unpk(acc) & 0xFFFFu) + (unpk(acc) >> 16);
			} else {
#pragma unroll
				for (uint32_t j = 0; j < EPT; j++)
					t += len_from_m<ENC, RICE>(half16(mp[c][j >> 1], j & 1u), s.cd);
			}
			T[c] = t;
#pragma unroll
			for (uint32_t i = 0; i < EPT / 2; i++) {
				asm volatile("" : "+v"(mp[c][i]));
				asm volatile("" : "+v"(mq[c][i]));
			}
		}
		uint32_t inc[NC];
#pragma unroll
		for (uint32_t c = 0; c < NC; c++) {
			inc[c] = wave_incl_scan(T[c]);
			if (lane == 63u)
				s_wsum[c][wid] = inc[c];
		}
		lds_barrier(); // wave totals and the code table visible; staging read
		// the staging area is free: the segment after this one streams in
		if (AIRS_PIPE_PF == 0 && wid == 3 && pf)
			pipe_prefetch<W, PRE>(a, pf_frame, pf_sif, lane, stage);
		s.A = 0u;
#pragma unroll
		for (uint32_t c = 0; c < NC; c++) {
			uint32_t woff = 0u, tt = 0u;
#pragma unroll
			for (uint32_t w = 0; w < EWG / 64; w++) {
				const uint32_t v = s_wsum[c][w];
				woff += w < wid ? v : 0u;
				tt += v;
			}
			excl[c] = woff + inc[c] - T[c];
			s.tot[c] = __builtin_amdgcn_readfirstlane(tt);
			s.A += s.tot[c];
		}
		const bool is_last = s.sif + 1u == a.segs_per_frame;
		if (!is_last && wid == EWG / 64 - 1) {
			// the segment's last 32 bits (lane 63 of the last wave): each lane's
			// stream tail, combined over four lanes (>= 64 bits)
			uint64_t acc = 0u;
			if (fastk) {
				const char *tab = reinterpret_cast<const char *>(s_rice[slot]);
				auto pair = [&](uint32_t j) {
#pragma unroll
					for (uint32_t h = 0; h < 2; h++) {
						const uint2 e = *reinterpret_cast<const uint2 *>(tab + half16(mq[NC - 1][j], h));
						acc = (acc << e.y) | (half16(mp[NC - 1][j], h) + e.x);
					}
				};
				if (s.cd.k >= 3u) { // >= 4 bits per sample: the last 8 samples hold >= 32 bits
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
					uint32_t c1, l1, c2, l2;
					code_from_m<ENC, RICE>(half16(mp[NC - 1][j >> 1], j & 1u), s.cd, c1, l1, c2, l2);
					acc = (acc << l1) | c1;
					if (NPIECE == 2)
						acc = (acc << l2) | c2;
				}
			}
			uint32_t v = (uint32_t)acc, tb = min(T[NC - 1], 32u);
#pragma unroll
			for (uint32_t dd = 1; dd <= 2; dd <<= 1) {
				const uint32_t va = __shfl_up(v, dd, 64), ta = __shfl_up(tb, dd, 64);
				if (lane >= dd && tb < 32u) {
					v = (va << tb) | v;
					tb = min(ta + tb, 32u);
				}
			}
			if (lane == 63u)
				gran_store(&a.tail[s.gseg], ((uint64_t)a.epoch << 32) | v);
		}
	};

	// the segment's aggregate (wave 0, lane 0): its bits, or for a frame's
	// first segment the inclusive prefix with the header
	auto publish_agg = [&](const PSeg<NC> &s) {
		if (lane == 0) {
			const bool f = s.sif == 0u;
			const uint64_t tag = ((uint64_t)a.epoch << 1) | (f ? 1u : 0u);
			gran_store(&a.agg[s.gseg], (tag << 32) | (f ? HDR_BITS + s.A : s.A));
		}
	};

	// ---- prologue: segment d_0 through phase 1, d_1's samples in flight ---
	const uint32_t d0 = blockIdx.x;
	if (AIRS_PIPE_PRIO) {
		const uint32_t slot = min(3u, (4u * d0) / G);
		if (slot == 1u)
			__builtin_amdgcn_s_setprio(1);
		else if (slot == 2u)
			__builtin_amdgcn_s_setprio(2);
		else if (slot == 3u)
			__builtin_amdgcn_s_setprio(3);
	}
	pseg_locate(a, d0, nfr, cur);
	if (wid == 3) {
		pipe_prefetch<W, PRE>(a, cur.frame, cur.sif, lane, stage);
		vm_wait();
	}
	bool has_next = d0 + G < a.num_segs;
	nxt = cur;
	if (has_next)
		pseg_locate(a, d0 + G, nfr, nxt);
	lds_barrier();
	phase1(cur, 0u, has_next, nxt.frame, nxt.sif);
	if (AIRS_PIPE_PF == 1 && wid == 3 && has_next)
		pipe_prefetch<W, PRE>(a, nxt.frame, nxt.sif, lane, stage);
	if (wid == 0)
		publish_agg(cur);

	for (;;) {
		const bool is_first = cur.sif == 0u;
		const bool is_last = cur.sif + 1u == a.segs_per_frame;
		pipe_stamp(a, cur.gseg, 0, tid);

		// ---- pack the chunks of `cur` into their images (bit 0 = chunk start)
#pragma unroll
		for (uint32_t c = 0; c < NC; c++) {
			uint32_t *Lc = imgs + c * IMGW + 4u;
			Packer pk1;
			pk1.init(Lc, excl[c]);
			if (cur.fastk) {
				const char *tab = reinterpret_cast<const char *>(s_rice[par]);
#pragma unroll
				for (uint32_t hb = 0; hb < 2; hb++) { // two batches of 8 lookups
					uint2 te[EPT / 2];
#pragma unroll
					for (uint32_t jj = 0; jj < EPT / 4; jj++) {
						const uint32_t j = hb * (EPT / 4) + jj;
#pragma unroll
						for (uint32_t h = 0; h < 2; h++)
							te[2 * jj + h] = *reinterpret_cast<const uint2 *>(tab + half16(mq[c][j], h));
					}
					uint32_t mxl = 0u;
#pragma unroll
					for (uint32_t i = 0; i < EPT / 2; i += 2)
						mxl = max(mxl, te[i].y + te[i + 1].y);
					if (__ballot(mxl > 32u) == 0ull) {
#pragma unroll
						for (uint32_t i = 0; i < EPT / 2; i += 2) {
							const uint32_t j = hb * (EPT / 2) + i;
							const uint32_t cwa = (mp[c][j >> 1] & 0xFFFFu) + te[i].x;
							const uint32_t cwb = (mp[c][j >> 1] >> 16) + te[i + 1].x;
							pk1.put((cwa << te[i + 1].y) | cwb, te[i].y + te[i + 1].y);
						}
					} else {
#pragma unroll
						for (uint32_t i = 0; i < EPT / 2; i += 2) {
							const uint32_t j = hb * (EPT / 2) + i;
							pk1.put((mp[c][j >> 1] & 0xFFFFu) + te[i].x, te[i].y);
							pk1.put((mp[c][j >> 1] >> 16) + te[i + 1].x, te[i + 1].y);
						}
					}
				}
			} else {
#pragma unroll
				for (uint32_t j = 0; j < EPT; j++) {
					uint32_t c1, l1, c2, l2;
					code_from_m<ENC, RICE>(half16(mp[c][j >> 1], j & 1u), cur.cd, c1, l1, c2, l2);
					pk1.put(c1, l1);
					if (NPIECE == 2)
						pk1.put(c2, l2);
				}
			}
			pk1.flush();
		}
		// the next segment's samples (DMA issued an iteration ago) land in the
		// staging area before the barrier
		if (wid == 3)
			vm_wait();
		lds_barrier(); // images complete, staging filled
		pipe_stamp(a, cur.gseg, 1, tid);

		// ---- look-back loads of `cur` (wave 0), evaluated after phase 1 ----
		uint64_t gv = 0ull, tv0 = 0ull;
		if (wid == 0) {
			const int64_t idx = (int64_t)cur.gseg - 1 - (int64_t)lane;
			gv = gran_issue(&a.agg[idx >= (int64_t)cur.first_seg ? idx : (int64_t)cur.first_seg]);
			tv0 = gran_issue(&a.tail[is_first ? cur.gseg : cur.gseg - 1u]);
		}

		// ---- phase 1 of the next segment, then its successor's prefetch ----
		const uint32_t npar = par ^ 1u;
		const bool pf = has_next && nxt.d + G < a.num_segs;
		PSeg<NC> n2 = nxt;
		if (has_next) {
			if (pf)
				pseg_locate(a, nxt.d + G, nfr, n2);
			phase1(nxt, npar, pf, n2.frame, n2.sif);
		}
		pipe_stamp(a, cur.gseg, 2, tid);

		// ---- look-back of `cur` (wave 0) ----------------------------------
		if (wid == 0) {
			vm_wait2(gv, tv0); // (the agg store below is issued after the wait)
			if (has_next)
				publish_agg(nxt);
			uint32_t Pw = HDR_BITS, pred;
			if (is_first) {
				// header bytes 20-21 (low half of the outlier field) share the
				// first payload dword of a 22-byte header
				pred = (EXT_HDR && ENC != ENC_RAW) ? (cur.cd.outlier & 0xFFFFu) : 0u;
			} else {
				uint32_t polls = 0u;
				Pw = pipe_lookback(a, cur.gseg, cur.first_seg, lane, gv, polls);
				if (lane == 0)
					gran_store(&a.agg[cur.gseg], ((((uint64_t)a.epoch << 1) | 1u) << 32) | (Pw + cur.A));
				uint64_t tv = tv0;
				uint32_t spins = 0;
				for (; (uint32_t)(tv >> 32) != a.epoch; spins++) {
					if (spins > AIRS_SPIN_LIMIT) {
						if (lane == 0)
							atomicAdd(a.ticket + AIRS_FAULT_WORD, 1u);
						break;
					}
					__builtin_amdgcn_s_sleep(1);
					tv = gran_fetch(&a.tail[cur.gseg - 1u]);
				}
				pred = (uint32_t)tv;
				if (AIRS_PIPE_TS && a.dbgts && lane == 0)
					a.dbgts[8u * cur.gseg + 6u] = (uint64_t)polls | ((uint64_t)spins << 32);
			}
			if (lane == 0) {
				s_misc[0] = Pw;
				s_misc[1] = pred;
			}
		}
		lds_barrier();
		const uint32_t P = __builtin_amdgcn_readfirstlane(s_misc[0]);
		pipe_stamp(a, cur.gseg, 3, tid);

		// ---- store the images, funnel-shifted to the frame bit offset (waves
		// 1-2; thread st = tid - 64) -----------------------------------------
		uint8_t *fdst = a.dst + (uint64_t)cur.frame * a.dst_stride;
		const uint32_t cap = a.cap;
		if (AIRS_PIPE_PF == 1 && wid == 3 && pf)
			pipe_prefetch<W, PRE>(a, n2.frame, n2.sif, lane, stage);
		if (wid == 1 || wid == 2) {
			const uint32_t st = tid - 64u;
			constexpr uint32_t NST = 128u;
			const __amdgpu_buffer_rsrc_t dst_rsrc =
				__builtin_amdgcn_make_buffer_rsrc(fdst, 0, (int)(cap & ~3u), 0x00020000);
			uint32_t base = 0u;
			uint32_t predx = st == 0u ? s_misc[1] : 0u; // (st 0) the 32 stream bits before chunk c
#pragma unroll
			for (uint32_t c = 0; c < NC; c++) {
				const uint32_t *Lx = imgs + c * IMGW + 4u;
				const lds_u32 *Ll = reinterpret_cast<const lds_u32 *>((uintptr_t)Lx);
				const uint32_t totx = cur.tot[c];
				const uint32_t Pc = P + base;
				const uint32_t r = Pc & 31u, g0 = Pc >> 5;
				const uint32_t endbit = Pc + totx;
				const uint32_t J = ((endbit - 1u) >> 5) - g0; // last word touched
				const uint32_t nfull = (endbit & 31u) == 0u ? J + 1u : J;
				const uint32_t nquad = nfull >> 2;
				for (uint32_t p = st; p < nquad; p += NST) {
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
				// the last nfull % 4 words: one each for the threads next in turn
				const uint32_t rr = (st + NST - nquad % NST) % NST;
				if (rr < (nfull & 3u)) {
					const uint32_t j = 4u * nquad + rr;
					const uint32_t hi = j ? Ll[j - 1u] : predx;
					const uint32_t v = __builtin_amdgcn_alignbit(hi, Ll[j], r);
					__builtin_amdgcn_raw_buffer_store_b32(bswap32(v), dst_rsrc, (int)(4u * (g0 + j)), 0, 0);
				}
				if (is_last && c == NC - 1u && nfull == J && st == 0u) {
					// zero-padded final bytes of the payload (reference bitstream_flush)
					const uint32_t hi = J ? Lx[J - 1u] : predx;
					const uint32_t v = __builtin_amdgcn_alignbit(hi, Lx[J], r);
					const uint32_t gw = g0 + J;
					const uint32_t nbytes = ((endbit & 31u) + 7u) >> 3;
					for (uint32_t b = 0; b < nbytes; b++)
						if (4u * gw + b < cap)
							fdst[4u * gw + b] = (uint8_t)(v >> (24u - 8u * b));
				}
				if (c + 1u < NC && st == 0u) {
					// the last 32 bits of this chunk precede the next (>= 4096 bits)
					const uint32_t s0 = totx - 32u, q = s0 >> 5, sh = s0 & 31u;
					predx = sh ? (Lx[q] << sh) | (Lx[q + 1] >> (32u - sh)) : Lx[q];
				}
				base += totx;
			}
		}

		// ---- frame epilogue (wave 0): checksum, header, status --------------
		if (is_last && tid == 0) {
			const uint32_t endbit = P + cur.A;
			const uint32_t payload_bytes = (endbit + 7u) >> 3;
			const uint32_t size = payload_bytes + (a.checksum ? 4u : 0u);
			if (a.checksum) {
				const uint32_t ck = sload32(a.checksums + cur.frame);
				for (uint32_t b = 0; b < 4u; b++)
					if (payload_bytes + b < cap)
						fdst[payload_bytes + b] = (uint8_t)(ck >> (24u - 8u * b));
			}
			const uint64_t id = a.ids ? sload64(a.ids + cur.lf) : a.id_base + (uint64_t)cur.lf * a.id_step;
			uint32_t h[5];
			header_words(h, size, 2u * a.n, id, a.seq, PRE, a.checksum ? 1u : 0u, ENC, 0u,
				     ENC == ENC_RAW ? 0u : cur.gpar, ENC == ENC_RAW ? 0u : cur.cd.outlier);
			const uint32_t hwords = EXT_HDR ? 5u : 4u;
#pragma unroll
			for (uint32_t w = 0; w < 5u; w++)
				if (w < hwords && 4u * w + 4u <= cap)
					*reinterpret_cast<uint32_t *>(fdst + 4u * w) = bswap32(h[w]);
			uint32_t stv = size;
			if (size > cap)
				stv = ERRV(E_DST_TOO_SMALL);
			else if (size > 0xFFFFFFu)
				stv = ERRV(E_HDR_CMP_SIZE_TOO_LARGE);
			a.status[cur.frame] = stv;
			if (a.needed)
				a.needed[cur.frame] = size;
		}
		pipe_stamp(a, cur.gseg, 4, tid);
		if (!has_next)
			break;

		// ---- clear the images for the next segment -------------------------
		lds_barrier(); // every store has read its words
#pragma unroll
		for (uint32_t c = 0; c < NC; c++) {
			uint32_t *Lc = imgs + c * IMGW + 4u;
			const uint32_t nw = (cur.tot[c] + 31u) >> 5;
			for (uint32_t i = tid; i <= nw; i += EWG)
				Lc[i] = 0u;
		}
		lds_barrier();
		pipe_stamp(a, cur.gseg, 5, tid);

		cur = nxt;
		par = npar;
		has_next = cur.d + G < a.num_segs;
		if (has_next)
			pseg_locate(a, cur.d + G, nfr, nxt);
	}
}

// ---------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------

template <int W, int PRE, int ENC, bool RICE>
static uint32_t pipe_go(const KArgs &k, hipStream_t s)
{
	auto kern = encode_pipe_kernel<W, PRE, ENC, RICE>;
	const size_t lds = (size_t)Stage<W>::BYTES + (size_t)pipe_chunks(W) * (k.img_words + 4u) * 4u;
	static int cus = 0;
	if (!cus) {
		int dev = 0;
		if (hipGetDevice(&dev) != hipSuccess ||
		    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
			return ERRV(E_GENERIC);
	}
	if (lds > 65536u) {
		static bool attr = false;
		if (!attr && hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
						 160 * 1024) != hipSuccess)
			return ERRV(E_GENERIC);
		attr = true;
	}
	int per_cu = 0;
	if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)kern, EWG, lds) != hipSuccess ||
	    per_cu <= 0)
		return ERRV(E_GENERIC);
	static int cap_env = -1;
	if (cap_env < 0) {
		const char *v = getenv("AIRS_PIPE_WGCU"); // experiments: workgroups per CU
		cap_env = v ? atoi(v) : 0;
	}
	if (cap_env > 0 && cap_env < per_cu)
		per_cu = cap_env;
	// the occupancy query can be one workgroup per CU high past 80 SGPRs
	// (MI355X_MICROARCH.md, residency): stay at or below 6, which the
	// hardware admits for any SGPR count this kernel uses
	per_cu = per_cu > 6 ? 6 : per_cu;
	const uint64_t resident = (uint64_t)per_cu * (uint64_t)cus;
	const uint64_t segs = k.num_segs;
	// balance the iterations: G <= resident, every workgroup the same count +- 1
	const uint64_t iters = (segs + resident - 1u) / resident;
	const uint32_t G = (uint32_t)((segs + iters - 1u) / iters);
	hipLaunchKernelGGL(kern, dim3(G), dim3(EWG), lds, s, k, G);
	return 0;
}

template <int W, int PRE>
static uint32_t pipe_enc(const KArgs &k, uint32_t enc, bool rice, hipStream_t s)
{
	switch (enc) {
	case ENC_RAW:
		return pipe_go<W, PRE, ENC_RAW, true>(k, s);
	case ENC_ZERO:
		return rice ? pipe_go<W, PRE, ENC_ZERO, true>(k, s) : pipe_go<W, PRE, ENC_ZERO, false>(k, s);
	default:
		return rice ? pipe_go<W, PRE, ENC_MULTI, true>(k, s) : pipe_go<W, PRE, ENC_MULTI, false>(k, s);
	}
}

uint32_t pipe_segn(uint32_t sample_bytes)
{
	return pipe_chunks(sample_bytes == 4 ? 4 : 2) * AIRS_SEG;
}

uint32_t pipe_encode(const KArgs &k, uint32_t sample_bytes, uint32_t pre, uint32_t enc, bool rice, hipStream_t s)
{
	if (sample_bytes == 2)
		return pre == PRE_DIFF ? pipe_enc<2, PRE_DIFF>(k, enc, rice, s) : pipe_enc<2, PRE_NONE>(k, enc, rice, s);
	return pre == PRE_DIFF ? pipe_enc<4, PRE_DIFF>(k, enc, rice, s) : pipe_enc<4, PRE_NONE>(k, enc, rice, s);
}

} // namespace airs
