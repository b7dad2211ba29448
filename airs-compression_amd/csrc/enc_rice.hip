// enc_rice.hip -- the Rice/ZERO frame kernel for 16-bit samples (gfx950):
// the encode hot path of BASELINE configs[1] and configs[3] (cfg2, cfg4).
//
// Same output as encode_kernel (enc_kernel.h), bit for bit: reference
// lib/compress/cmp.c:296-312 (per-sample loop), NONE/DIFF residuals
// preprocess.c:268-300, ZigZag encoder.c:274-286, Golomb ZERO with g = 2^k
// encoder.c:327-351 (zero escape :340-346), big-endian bit packing
// bitstream_writer.h:124-158 with its flush :205-227, header header.c:24-67,
// checksum header.c:137-163.  Eligible: 16-bit samples, NONE or DIFF,
// GOLOMB_ZERO with g = 2^k, k <= RICE_KMAX, no model, whole 16 Ki-sample
// segments, 16-byte aligned frames.
//
// What differs from encode_kernel is how much of the chip a segment holds
// while it waits:
//   * phase 1 turns every sample pair into its final codeword pair V (one
//     32-bit register: the two codewords back to back) and its length L
//     (four lengths per register), instead of keeping the mapped values AND
//     the code-table offsets: 40 registers per lane for the segment's 64
//     samples instead of 64.  The table lookups move into phase 1, where
//     they overlap the sample loads of the other workgroups; the packer
//     reads no LDS at all.  Round 6: one lookup per PAIR, in a table of
//     the 18 x 18 (min(q_a, 17), min(q_b, 17)) combinations holding
//     P = (T'[q_a] << l_b) + T'[q_b] and the lengths, so that V =
//     (m_a << l_b) + m_b + P (15 VALU per pair instead of 18, 65 VGPRs
//     instead of 80; six workgroups per CU);
//   * the segment is packed back to back into ONE arena sized for a
//     compressed segment (~11 bits per sample at six workgroups per CU; a
//     segment that does not fit is packed and stored chunk by chunk), so
//     there is no image rotation: three barriers per segment (encode_kernel:
//     seven);
//   * the look-back is evaluated once the whole segment is packed, so its
//     predecessors published their aggregates long before (no retries); for
//     frames whose segments all run on one XCD its polls are scalar loads
//     (rice_lookback_s).
// AUTO (cfg3): the frame's k is chosen in the kernel from a histogram and a
// candidate barrier (rice_auto_k) before phase 1; no look-back.
// A pair whose two codewords exceed 32 bits (two zero escapes, or one
// escape next to a long code) keeps its mapped values in V; the packer
// re-codes it from the table in a wave-uniform slow step.
//
// Look-back granules, frame-interleaved dispatch, the tail granule and the
// bounded spins are those of encode_kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "enc_common.h"

namespace airs {

#ifndef AIRS_RICE_WG // threads per workgroup (256 or 512)
#define AIRS_RICE_WG 256
#endif
// workgroups per CU the LDS arena (and the register allocation) is sized
// for: DIFF and NONE frames 6 (round 6: with the scalar look-back the chains
// no longer stall at more than four; cfg2 53.0-53.9 -> 50.1-53.5 us, with
// the nt stores 47.8-51.2; the pair table took the kernel from 80 to 65
// VGPRs, and 7 or 8 per CU measured the same as 6), AUTO 5 (its mapped
// samples stay live across the candidate barrier; 62 VGPRs since the
// barrier polls one granule per lane at a time, 99 before; 5 beat 4 and 6)
#ifndef AIRS_RICE_WGPCU
#define AIRS_RICE_WGPCU 6
#endif
#ifndef AIRS_RICE_NONE_WGPCU
#define AIRS_RICE_NONE_WGPCU 6
#endif
#ifndef AIRS_RICE_AUTO_WGPCU
#define AIRS_RICE_AUTO_WGPCU 5
#endif
// AUTO histogram counters per bin: 64 (one per lane) or 32 (lanes l and
// l + 32 share one, two-way atomic conflicts: half the LDS, so that the
// histogram fits the arena of five workgroups per CU)
#ifndef AIRS_RICE_AUTO_HCOLS
#define AIRS_RICE_AUTO_HCOLS 32
#endif
#ifndef AIRS_RICE_LBC // the look-back is evaluated after packing this many chunks (wave 0)
#define AIRS_RICE_LBC 4
#endif
#ifndef AIRS_RICE_SLB // granules of the scalar first look-back round (16 or 32)
#define AIRS_RICE_SLB 16
#endif
// cache policy of the payload stores (gfx950 aux: 2 = nt): the output is
// written once and not read back by this kernel (round 6: a 128 MiB read +
// 56 MiB dense write stream 34.3 -> 32.2 us, scripts/stream_bench.hip)
#ifndef AIRS_RICE_STORE_AUX
#define AIRS_RICE_STORE_AUX 2
#endif
#define RICE_KMAX 7u       // largest k this kernel takes (pairs of typical codes fit 32 bits)
constexpr uint32_t RWG = AIRS_RICE_WG;      // threads per workgroup
constexpr uint32_t RNW = RWG / 64u;         // waves per workgroup
constexpr uint32_t RCHUNK = RWG * 16u;      // samples per chunk: lane t owns [16t, 16t+16)
constexpr uint32_t RCH = 4u;                // chunks per segment
constexpr uint32_t RSEGN = RCH * RCHUNK;    // samples per segment (16 Ki or 32 Ki)
constexpr uint32_t RGUARD = 4u;              // words before the arena (a lane's first put ORs zeros there)
// LDS per workgroup is allocated in granules: leave room for the static LDS
// and the rounding (measured: a 32464-byte workgroup admitted only four per CU)
constexpr uint32_t RSTATIC = 2048u + 18u * 18u * 8u; // (+ the pair table)

template <int PRE, bool AUTO>
__host__ __device__ constexpr uint32_t rice_wgpcu()
{
	return AUTO ? AIRS_RICE_AUTO_WGPCU : PRE == PRE_NONE ? AIRS_RICE_NONE_WGPCU : AIRS_RICE_WGPCU;
}

// arena words (guard included) for `wgpcu` workgroups per CU
__host__ __device__ constexpr uint32_t rice_arena_words(uint32_t wgpcu)
{
	return ((160u * 1024u / wgpcu - RSTATIC) / 4u) & ~3u;
}

// the four words of a lane's chunk: lengths of pairs 4h .. 4h+3, a byte each
__device__ __forceinline__ uint32_t len_byte(const uint32_t (&lp)[2], uint32_t j)
{
	const uint32_t w = lp[j >> 2], b = j & 3u;
	return b == 0u ? (w & 0xFFu) : b == 3u ? (w >> 24) : ((w >> (8u * b)) & 0xFFu);
}

// (codeword, length) of one mapped value from the table (slow steps only)
__device__ __forceinline__ uint2 rice_code(uint32_t m, uint32_t k, const uint2 *tab)
{
	const uint32_t q = (m + 1u) >> k;
	const uint2 e = tab[q < 17u ? q : 17u];
	return make_uint2(m + e.x, e.y);
}

// Bit packer of one lane into the arena (as enc_common.h Packer): nb is the
// bit position in the LDS address space less 32, acc the last bits.
struct RPack {
	uint64_t acc;
	uint32_t nb;
	__device__ __forceinline__ void init(uint32_t bitaddr)
	{
		acc = 0u;
		nb = bitaddr - 32u;
	}
	__device__ __forceinline__ void put(uint32_t v, uint32_t len) // len <= 32, v < 2^len
	{
		acc = (acc << len) | v;
		nb += len;
		lds_u32 *w = reinterpret_cast<lds_u32 *>((uintptr_t)((nb >> 3) & ~3u));
		__hip_atomic_fetch_or(w, __builtin_amdgcn_alignbit((uint32_t)(acc >> 32), (uint32_t)acc, nb),
				      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
	}
	__device__ __forceinline__ void flush()
	{
		if (nb & 31u) {
			lds_u32 *w = reinterpret_cast<lds_u32 *>((uintptr_t)(((nb >> 3) & ~3u) + 4u));
			__hip_atomic_fetch_or(w, (uint32_t)acc << (32u - (nb & 31u)), __ATOMIC_RELAXED,
					      __HIP_MEMORY_SCOPE_WORKGROUP);
		}
	}
};

// Pack one lane's 8 pairs of a chunk.  Pairs of more than 32 bits hold their
// mapped values in V (the two halves) and are re-coded here; the test is one
// ballot per chunk, then one per pair inside chunks that have such a pair.
__device__ __forceinline__ void pack_chunk(RPack &p, const uint32_t (&V)[8], const uint32_t (&lp)[2], uint32_t k,
					   const uint2 *tab)
{
	const uint32_t ov = ((lp[0] + 0x1F1F1F1Fu) | (lp[1] + 0x1F1F1F1Fu)) & 0x40404040u; // some L > 32
	if (__ballot(ov != 0u) == 0ull) {
#pragma unroll
		for (uint32_t j = 0; j < 8u; j++)
			p.put(V[j], len_byte(lp, j));
		return;
	}
#pragma unroll
	for (uint32_t j = 0; j < 8u; j++) {
		const uint32_t L = len_byte(lp, j);
		if (__ballot(L > 32u) == 0ull) {
			p.put(V[j], L);
		} else {
			const bool big = L > 32u;
			const uint2 ca = rice_code(V[j] & 0xFFFFu, k, tab), cb = rice_code(V[j] >> 16, k, tab);
			p.put(big ? ca.x : 0u, big ? ca.y : 0u);
			p.put(big ? cb.x : V[j], big ? cb.y : L);
		}
	}
}

// Evaluate a look-back from a first window (gv: granule gseg - 1 - lane,
// newest first; tv: the predecessor's tail granule), reloading with vector
// loads until the segment's frame bit offset is known: (offset, the
// predecessor's last 32 bits).  Every published granule stays true, so the
// first window may be of any age.
__device__ __forceinline__ uint2 lb_resolve(const KArgs &a, uint32_t gseg, uint32_t sif, uint32_t lane, uint64_t gv,
					    uint64_t tv, uint32_t rounds)
{
	const uint32_t first_seg = gseg - sif;
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
		if (!(bad_m & need)) {
			sum += wave_sum((inr && lane <= fi) ? (uint32_t)gv : 0u);
			if (incl_m)
				break;
			j -= 64; // every granule of this window is an aggregate: the next window
			rounds++;
		} else if (++spins > AIRS_SPIN_LIMIT) {
			if (lane == 0)
				atomicAdd(a.ticket + AIRS_FAULT_WORD, 1u); // never expected (the host reports it)
			break;
		} else {
			__builtin_amdgcn_s_sleep(1); // a needed predecessor has not published: re-poll
			rounds++;
		}
		const int64_t nidx = j - (int64_t)lane;
		gv = gran_load(&a.agg[nidx >= (int64_t)first_seg ? nidx : (int64_t)first_seg]);
	}
	// the predecessor's tail (lane 0's copy is the one used)
	uint32_t s2 = 0;
	for (; (uint32_t)(tv >> 32) != a.epoch; s2++) {
		if (s2 > AIRS_SPIN_LIMIT) {
			if (lane == 0)
				atomicAdd(a.ticket + AIRS_FAULT_WORD, 1u);
			break;
		}
		__builtin_amdgcn_s_sleep(1);
		tv = gran_load(&a.tail[gseg - 1u]);
	}
	if (DBG(65536u) && !DBG(262144u) && a.dbgts && lane == 0) {
		a.dbgts[8u * gseg + 5u] = ((uint64_t)spins << 32) | rounds;
		a.dbgts[8u * gseg + 6u] = s2;
	}
	return make_uint2(sum, (uint32_t)tv);
}

// The look-back (wave 0): the segment's frame bit
// offset P (header bits included) and the predecessor's last 32 bits.  The
// first round reads the 16 newest granules and the tail through scalar loads
// (one asm statement with its wait: no register of an outstanding load is
// visible to the compiler); further rounds are vector loads of
// 64 granules, newest first.  Not for the frame's first segment.
__device__ __forceinline__ uint2 rice_lookback(const KArgs &a, uint32_t gseg, uint32_t sif, uint32_t lane,
					       uint64_t gearly)
{
	uint32_t rounds = 1u;
	constexpr uint32_t SLB_N = AIRS_RICE_SLB;
	const uint32_t first_seg = gseg - sif;
	uint64_t gv = 0ull, tv = 0ull;
	bool have = false;
	if (sif >= SLB_N) {
		typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
		auto sptr = [](const uint64_t *p) {
			const uint64_t v = (uint64_t)(uintptr_t)p;
			const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)v);
			const uint32_t h = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
			return (const uint64_t *)(uintptr_t)(((uint64_t)h << 32) | l);
		};
		const uint64_t *gp = sptr(&a.agg[gseg - SLB_N]);
		const uint64_t *tp = sptr(&a.tail[gseg - 1u]);
		// q[b]: granules gseg - SLB_N + 8 b .. + 7 -> lanes SLB_N - 1 - (8 b + i);
		// lanes >= SLB_N read as unpublished
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
		else
			asm volatile("s_load_dwordx16 %0, %3, 0x0 glc\n\t"
				     "s_load_dwordx16 %1, %3, 0x40 glc\n\t"
				     "s_load_dwordx2 %2, %4, 0x0 glc\n\t"
				     "s_waitcnt lgkmcnt(0)"
				     : "=&s"(q[0]), "=&s"(q[1]), "=&s"(tq)
				     : "s"(gp), "s"(tp)
				     : "memory");
		// lanes >= SLB_N: the window read when the aggregate was published
		// (granules gseg - 1 - lane; any published value stays true)
		uint32_t vl = (uint32_t)gearly, vh = (uint32_t)(gearly >> 32);
#pragma unroll
		for (uint32_t i = 0; i < SLB_N; i++) {
			vl = lane == SLB_N - 1u - i ? q[i >> 3][2u * (i & 7u)] : vl;
			vh = lane == SLB_N - 1u - i ? q[i >> 3][2u * (i & 7u) + 1u] : vh;
		}
		gv = ((uint64_t)vh << 32) | vl;
		tv = tq;
		have = true;
	}
	if (!have) {
		const int64_t idx = (int64_t)gseg - 1 - (int64_t)lane;
		gv = gran_load(&a.agg[idx >= (int64_t)first_seg ? idx : (int64_t)first_seg]);
		tv = gran_load(&a.tail[gseg - 1u]);
	}
	return lb_resolve(a, gseg, sif, lane, gv, tv, rounds);
}

// The look-back on scalar loads only (lbmode bit 0: a frame's segments all
// run on one XCD, so its L2 holds every granule the frame's segments write
// and a scalar load that misses the scalar cache sees the newest value).
// A vector poll queues behind the CU's sample loads (~2.4 us per re-poll on
// a loaded CU); a scalar poll does not (~1 us).  Windows of
// 16 granules, newest first, evaluated in scalar code: granules are summed
// down to the nearest inclusive one; an unpublished granule is re-polled
// after s_sleep, with the sum of the newer ones kept; a window of aggregates
// only moves on to the next one at once.  After AIRS_RICE_SPOLL polls the
// vector look-back takes over (liveness whatever the placement).  sif >= 16.
#ifndef AIRS_RICE_SPOLL
#define AIRS_RICE_SPOLL 4096u
#endif
#ifndef AIRS_RICE_SWIN // granules per scalar window (8: one s_load_dwordx16; 16: two)
#define AIRS_RICE_SWIN 16
#endif
__device__ __forceinline__ uint2 rice_lookback_s(const KArgs &a, uint32_t gseg, uint32_t sif, uint32_t lane)
{
	typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
	constexpr uint32_t SW = AIRS_RICE_SWIN;
	auto sptr = [](const uint64_t *p) {
		const uint64_t v = (uint64_t)(uintptr_t)p;
		const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)v);
		const uint32_t h = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
		return (const uint64_t *)(uintptr_t)(((uint64_t)h << 32) | l);
	};
	const uint32_t first_seg = gseg - sif, epoch = a.epoch;
	uint32_t sum = 0u, polls = 0u, rounds = 0u, j = gseg - 1u;
	uint64_t tv = 0ull;
	bool have_tail = false, done = false;
	while (polls < AIRS_RICE_SPOLL) {
		const uint32_t base = j >= first_seg + (SW - 1u) ? j - (SW - 1u) : first_seg;
		const uint64_t *gp = sptr(&a.agg[base]);
		u32x16 q[SW / 8u];
		if (!have_tail) {
			const uint64_t *tp = sptr(&a.tail[gseg - 1u]);
			if constexpr (SW == 16u)
				asm volatile("s_load_dwordx16 %0, %3, 0x0 glc\n\t"
					     "s_load_dwordx16 %1, %3, 0x40 glc\n\t"
					     "s_load_dwordx2 %2, %4, 0x0 glc\n\t"
					     "s_waitcnt lgkmcnt(0)"
					     : "=&s"(q[0]), "=&s"(q[SW / 8u - 1u]), "=&s"(tv)
					     : "s"(gp), "s"(tp)
					     : "memory");
			else
				asm volatile("s_load_dwordx16 %0, %2, 0x0 glc\n\t"
					     "s_load_dwordx2 %1, %3, 0x0 glc\n\t"
					     "s_waitcnt lgkmcnt(0)"
					     : "=&s"(q[0]), "=&s"(tv)
					     : "s"(gp), "s"(tp)
					     : "memory");
			have_tail = (uint32_t)(tv >> 32) == epoch;
		} else {
			if constexpr (SW == 16u)
				asm volatile("s_load_dwordx16 %0, %2, 0x0 glc\n\t"
					     "s_load_dwordx16 %1, %2, 0x40 glc\n\t"
					     "s_waitcnt lgkmcnt(0)"
					     : "=&s"(q[0]), "=&s"(q[SW / 8u - 1u])
					     : "s"(gp)
					     : "memory");
			else
				asm volatile("s_load_dwordx16 %0, %1, 0x0 glc\n\t"
					     "s_waitcnt lgkmcnt(0)"
					     : "=&s"(q[0])
					     : "s"(gp)
					     : "memory");
		}
		rounds++;
		// newest first: 0 = every granule an aggregate, 1 = inclusive found,
		// 2 = granule `j` unpublished
		uint32_t stop = 0u;
#pragma unroll
		for (int i = (int)SW - 1; i >= 0; i--) {
			const uint32_t lo = q[i >> 3][2 * (i & 7)], hi = q[i >> 3][2 * (i & 7) + 1];
			if (stop == 0u && base + (uint32_t)i <= j) {
				if ((hi >> 1) != epoch) {
					stop = 2u;
					j = base + (uint32_t)i;
				} else {
					sum += lo;
					stop = hi & 1u;
				}
			}
		}
		if (stop == 1u) {
			done = true;
			break;
		}
		if (stop == 0u) {
			if (base == first_seg) // never: the frame's first granule is inclusive
				break;
			j = base - 1u;
			continue;
		}
		polls++;
		__builtin_amdgcn_s_sleep(1);
	}
	// the predecessor's tail
	while (done && !have_tail && polls < AIRS_RICE_SPOLL) {
		const uint64_t *tp = sptr(&a.tail[gseg - 1u]);
		polls++;
		__builtin_amdgcn_s_sleep(1);
		asm volatile("s_load_dwordx2 %0, %1, 0x0 glc\n\t"
			     "s_waitcnt lgkmcnt(0)"
			     : "=&s"(tv)
			     : "s"(tp)
			     : "memory");
		have_tail = (uint32_t)(tv >> 32) == epoch;
	}
	if (DBG(65536u) && !DBG(262144u) && a.dbgts && lane == 0) {
		a.dbgts[8u * gseg + 5u] = ((uint64_t)polls << 32) | rounds;
		a.dbgts[8u * gseg + 6u] = 0u;
	}
	if (done && have_tail)
		return make_uint2(sum, (uint32_t)tv);
	// the vector look-back from the start (never expected on one XCD)
	const int64_t idx = (int64_t)gseg - 1 - (int64_t)lane;
	const uint64_t gv = gran_load(&a.agg[idx >= (int64_t)first_seg ? idx : (int64_t)first_seg]);
	return lb_resolve(a, gseg, sif, lane, gv, gran_load(&a.tail[gseg - 1u]), rounds);
}

// Store `tot` bits of an LDS image (bit 0 of word 0 = bit Pc of the frame)
// to the frame: each complete word funnel-shifted to Pc mod 32, byte-swapped,
// written through the frame's buffer descriptor (range = capacity rounded
// down to words, so the hardware drops what does not fit); the final partial
// word as bytes when `finalx` (reference bitstream_flush).  As
// encode_kernel's store_chunk.
__device__ __forceinline__ void rice_store(const uint32_t *Lx, uint32_t Pc, uint32_t totx, uint32_t predx, bool finalx,
					   __amdgpu_buffer_rsrc_t rsrc, uint8_t *fdst, uint32_t cap, uint32_t tid)
{
	if (!totx)
		return;
	const uint32_t r = Pc & 31u, g0 = Pc >> 5;
	const uint32_t endbit = Pc + totx;
	const uint32_t J = ((endbit - 1u) >> 5) - g0;
	const uint32_t nfull = (endbit & 31u) == 0u ? J + 1u : J;
	const lds_u32 *Ll = reinterpret_cast<const lds_u32 *>((uintptr_t)Lx);
	const uint32_t nquad = nfull >> 2;
	for (uint32_t p = tid; p < nquad; p += RWG) {
		const uint32_t j = 4u * p;
		const u32x4 w = *reinterpret_cast<const __attribute__((address_space(3))) u32x4 *>(Ll + j);
		const uint32_t hi = j ? Ll[j - 1u] : predx;
		u32x4 o;
		o.x = bswap32(__builtin_amdgcn_alignbit(hi, w.x, r));
		o.y = bswap32(__builtin_amdgcn_alignbit(w.x, w.y, r));
		o.z = bswap32(__builtin_amdgcn_alignbit(w.y, w.z, r));
		o.w = bswap32(__builtin_amdgcn_alignbit(w.z, w.w, r));
		__builtin_amdgcn_raw_buffer_store_b128(o, rsrc, (int)(4u * (g0 + j)), 0, AIRS_RICE_STORE_AUX);
	}
	const uint32_t rr = (tid - nquad) & (RWG - 1u);
	if (rr < (nfull & 3u)) {
		const uint32_t j = 4u * nquad + rr;
		const uint32_t hi = j ? Ll[j - 1u] : predx;
		__builtin_amdgcn_raw_buffer_store_b32(bswap32(__builtin_amdgcn_alignbit(hi, Ll[j], r)), rsrc,
						      (int)(4u * (g0 + j)), 0, AIRS_RICE_STORE_AUX);
	}
	if (finalx && nfull == J && tid == 0) {
		const uint32_t hi = J ? Lx[J - 1u] : predx;
		const uint32_t v = __builtin_amdgcn_alignbit(hi, Lx[J], r);
		const uint32_t gw = g0 + J;
		const uint32_t nbytes = ((endbit & 31u) + 7u) >> 3;
		for (uint32_t b = 0; b < nbytes; b++)
			if (4u * gw + b < cap)
				fdst[4u * gw + b] = (uint8_t)(v >> (24u - 8u * b));
	}
}

// AUTO: the predecessor's last 32 bits (its tail granule, published once it
// knows the frame's k), polled by wave 0 (bounded as every wait)
__device__ __forceinline__ uint32_t rice_tail_wait(const KArgs &a, uint32_t gseg)
{
	uint64_t tv = gran_load(&a.tail[gseg - 1u]);
	for (uint32_t s2 = 0; (uint32_t)(tv >> 32) != a.epoch; s2++) {
		if (s2 > AIRS_SPIN_LIMIT) {
			if ((threadIdx.x & 63u) == 0)
				atomicAdd(a.ticket + AIRS_FAULT_WORD, 1u);
			break;
		}
		__builtin_amdgcn_s_sleep(1);
		tv = gran_load(&a.tail[gseg - 1u]);
	}
	return (uint32_t)tv;
}

// AUTO (CMP_GPU_AUTO_RICE, fused): the frame's k and this segment's payload
// bit offset (header excluded), from the mapped pairs mp, as encode_kernel's
// AUTO (enc_kernel.h): a 129-bin histogram of v = m + 1 in
// the (zeroed) arena, one 32-bit counter per (bin, lane) shared by the four
// waves (bank = lane); the bin totals; the segment's 16 candidate sums
// S_k = sum min(v >> k, 16), published as epoch-tagged granules; wave 0
// reads the frame's spf * 16 granules (the frame barrier), takes the k with
// the fewest bits n (k + 1) + S_k (ties to the smaller k) and the sum of
// S_k over the segments before this one.  Leaves the arena zero again.
__device__ __forceinline__ uint2 rice_auto_k(const KArgs &a, uint32_t *H, uint32_t (&mp)[RCH][8], uint32_t gseg, uint32_t sif,
			     uint32_t tid, uint32_t lane, uint32_t wid)
{
	__shared__ uint32_t s_hist[AUTO_BINS];
	__shared__ uint32_t s_kt[RNW][16];
	__shared__ uint32_t s_res[2];
	// this lane's counter of bin b is at byte hbase + 4 HC (b + 1016): the
	// bin's offset comes from the float bits with one shift and one shift-add
	// (the 32-bit LDS address arithmetic wraps)
	constexpr uint32_t HC = AIRS_RICE_AUTO_HCOLS, HSH = HC == 64u ? 8u : 7u;
	static_assert(HC == 64u || HC == 32u, "64 or 32 counters per bin");
	const uint32_t hbase = (uint32_t)(uintptr_t)H + 4u * (lane & (HC - 1u)) - 1016u * 4u * HC;
	__syncthreads(); // the arena is zeroed
#pragma unroll
	for (uint32_t c = 0; c < RCH; c++) {
#pragma unroll
		for (uint32_t jp = 0; jp < 8u; jp++) {
			// the pair made opaque in place (no copy): otherwise the compiler
			// computes all 64 bins ahead of the barrier above
			asm volatile("" : "+v"(mp[c][jp]));
			const uint32_t wv = mp[c][jp];
#pragma unroll
			for (uint32_t h = 0; h < 2; h++) {
				const uint32_t v = (h ? wv >> 16 : wv & 0xFFFFu) + 1u;
				uint32_t ha;
				asm("v_lshrrev_b32 %0, 20, %1\n\tv_lshl_add_u32 %0, %0, %3, %2"
				    : "=&v"(ha)
				    : "v"(__float_as_uint((float)v)), "v"(hbase), "i"(HSH));
				__hip_atomic_fetch_add(reinterpret_cast<lds_u32 *>((uintptr_t)ha), 1u, __ATOMIC_RELAXED,
						       __HIP_MEMORY_SCOPE_WORKGROUP);
			}
		}
	}
	__syncthreads();
	// bin totals: threads 2r, 2r + 1 sum the halves of row r < 128 with
	// HC / 8 16-byte reads each, rotated by r (bank sharing); wave 0 row 128
	{
		constexpr uint32_t NQ = HC / 8u; // 16-byte reads per half row
		const uint32_t r = tid >> 1, h = tid & 1u;
		const uint4 *row = reinterpret_cast<const uint4 *>(H + r * HC + h * (HC / 2u));
		uint32_t sm = 0u;
#pragma unroll
		for (uint32_t hq = 0; hq < NQ; hq += 4u) {
			uint4 q4[4];
#pragma unroll
			for (uint32_t q = 0; q < 4u; q++)
				q4[q] = row[(hq + q + r) & (NQ - 1u)];
#pragma unroll
			for (uint32_t q = 0; q < 4u; q++)
				sm += q4[q].x + q4[q].y + q4[q].z + q4[q].w;
		}
		sm += __shfl_xor(sm, 1, 64);
		if (h == 0u)
			s_hist[r] = sm;
		static_assert(RWG != 256u || AUTO_BINS == RWG / 2u + 1u, "rows 0..127 by thread pairs, then row 128");
		if (wid == 0) {
			const uint32_t s128 = wave_sum(lane < HC ? H[128u * HC + lane] : 0u);
			if (lane == 0)
				s_hist[128] = s128;
		}
	}
	__syncthreads();
	// the arena again as the arena: clear the histogram rows
	for (uint32_t i = tid; i < AUTO_BINS * HC / 4u; i += RWG)
		reinterpret_cast<uint4 *>(H)[i] = make_uint4(0u, 0u, 0u, 0u);
	// the segment's 16 candidate sums: thread (slice sl, k) covers bins sl,
	// sl + 16, ...; the four slices of a wave meet through two shuffles.
	// auto_term without branches: bin b = 8 t + f (top bit t, next three
	// bits f) and x = (8 + f) << 4; min(v >> k, 16) summed over the bin is
	// min(16, x >> max(k + 7 - t, 0)): 16 when k <= t - 4, 0 when k > t, the
	// top t - k + 1 bits otherwise.  f is the thread's (sl mod 8), t grows by
	// 2 per step.
	{
		const uint32_t k = tid & 15u, sl = tid >> 4;
		const uint32_t x = (8u + (sl & 7u)) << 4;
		const int32_t sh0 = (int32_t)k + 7 - (int32_t)(sl >> 3);
		uint32_t part = 0u;
#pragma unroll
		for (uint32_t i = 0; i < (AUTO_BINS + 15u) / 16u; i++) {
			const uint32_t b = sl + 16u * i;
			const uint32_t term = min(16u, x >> (uint32_t)max(sh0 - 2 * (int32_t)i, 0));
			if (i + 1u < (AUTO_BINS + 15u) / 16u || b < AUTO_BINS)
				part += __umul24(s_hist[b < AUTO_BINS ? b : 0u], b < AUTO_BINS ? term : 0u); // (< 2^14 x 16)
		}
		part += __shfl_xor(part, 16, 64);
		part += __shfl_xor(part, 32, 64);
		if (lane < 16u)
			s_kt[wid][k] = part;
	}
	__syncthreads();
	if (wid == 0) {
		// publish (lanes 0-15), then read the frame's 16 * spf granules
		if (lane < 16u) {
			uint32_t sk = 0u;
#pragma unroll
			for (uint32_t w = 0; w < RNW; w++)
				sk += s_kt[w][lane];
			gran_store(&a.ktot[(uint64_t)gseg * 16u + lane], ((uint64_t)a.epoch << 32) | sk);
		}
		dbg_stamp(a, gseg, 5); // (AUTO: candidates published)
		const uint32_t first_seg = gseg - sif, ng = a.segs_per_frame * 16u;
		// 64 granules per round (one per lane), the rounds one after another
		// so that no window of granules stays live beside the mapped pairs
		// (cfg3's frames: one round)
		uint32_t tot = 0u, pre = 0u, spins = 0u;
		const uint32_t nit = (ng + 63u) / 64u;
		for (uint32_t i = 0; i < nit; i++) {
			const uint32_t gi = 64u * i + lane;
			const uint64_t *gp = &a.ktot[(uint64_t)first_seg * 16u + (gi < ng ? gi : 0u)];
			uint64_t g = gran_load(gp);
			for (;;) {
				const bool bad = gi < ng && (uint32_t)(g >> 32) != a.epoch;
				if (!__ballot(bad))
					break;
				if (++spins > AIRS_SPIN_LIMIT) {
					if (lane == 0)
						atomicAdd(a.ticket + AIRS_FAULT_WORD, 1u);
					break;
				}
				__builtin_amdgcn_s_sleep(1);
				if (bad)
					g = gran_load(gp);
			}
			// lane l holds segment 4 i + l / 16, candidate k = l % 16
			const uint32_t v = gi < ng ? (uint32_t)g : 0u;
			tot += v;
			pre += (gi >> 4) < sif ? v : 0u;
		}
		dbg_stamp(a, gseg, 6); // (AUTO: every candidate of the frame seen)
		tot += __shfl_xor(tot, 16, 64);
		tot += __shfl_xor(tot, 32, 64);
		pre += __shfl_xor(pre, 16, 64);
		pre += __shfl_xor(pre, 32, 64);
		const uint32_t k = lane & 15u;
		// frame bits for k (< 2^28: spf <= 32 segments), ties to the smaller k
		uint32_t key = ((tot + a.n * (k + 1u)) << 4) | k;
#pragma unroll
		for (uint32_t dd = 1; dd < 16u; dd <<= 1)
			key = min(key, (uint32_t)__shfl_xor(key, dd, 64));
		const uint32_t ks = key & 15u;
		const uint32_t pre_k = __shfl(pre, ks, 64);
		if (lane == 0) {
			s_res[0] = ks;
			s_res[1] = pre_k + sif * RSEGN * (ks + 1u); // every segment before this one is whole
		}
	}
	__syncthreads();
	return make_uint2(__builtin_amdgcn_readfirstlane(s_res[0]), __builtin_amdgcn_readfirstlane(s_res[1]));
}

// The pair table (rice_kernel's s_ptab) for k: 324 entries by the whole
// workgroup (before B0)
__device__ __forceinline__ void rice_pair_table(uint2 *pt, uint32_t k, uint32_t tid)
{
	// T'[q] in 32 bits (q + k <= 31: 2 << 31 wraps to the right residue)
	auto ent = [k](uint32_t q) {
		return q >= 17u ? make_uint2(0u, k + 17u)
				: make_uint2((2u << (q + k)) - (2u << k) - (q << k) + 1u, k + 1u + q);
	};
	for (uint32_t i = tid; i < 18u * 18u; i += RWG) {
		const uint32_t qa = __umul24(i, 3641u) >> 16, qb = i - 18u * qa; // (i / 18 for i < 324)
		const uint2 ea = ent(qa), eb = ent(qb);
		// (mod 2^32; exact when L <= 32, meaningless otherwise, e.g. l_b = 32)
		pt[i] = make_uint2((ea.x << (eb.y & 31u)) + eb.x, eb.y | ((ea.y + eb.y) << 8));
	}
}

// the lane's samples of segment `sif` of a frame: 4 chunks x 16 samples, and
// for DIFF the sample before each chunk's first (lane 0 of each wave uses it;
// every lane loads, so the load needs no branch; 0 before the frame's first
// sample, reference preprocess.c:268-300)
template <int PRE>
__device__ __forceinline__ void rice_load(const KArgs &a, const uint8_t *fsrc, uint32_t sif, uint32_t gseg, uint32_t tid,
					  uint4 (&raw)[RCH][2], uint32_t (&prevld)[RCH])
{
#pragma unroll
	for (uint32_t c = 0; c < RCH; c++) {
		const uint32_t first = sif * RSEGN + c * RCHUNK + tid * EPT;
		const uint4 *p = reinterpret_cast<const uint4 *>(fsrc + (size_t)first * 2u);
		if (DBG(512u)) { // ablation: no HBM reads (noise of width ~64 made in registers)
			uint32_t h = (first * 2654435761u) ^ (gseg * 40503u);
			uint32_t wv[8];
#pragma unroll
			for (uint32_t q = 0; q < 8u; q++) {
				h = h * 1664525u + 1013904223u;
				wv[q] = 0x40004000u + ((h >> 8) & 0x003F003Fu);
			}
			raw[c][0] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
			raw[c][1] = make_uint4(wv[4], wv[5], wv[6], wv[7]);
		} else {
			raw[c][0] = p[0];
			raw[c][1] = p[1];
		}
		// (the caller zeroes it for the frame's first sample, at the use:
		// a select here would make the compiler wait for the load)
		if (PRE == PRE_DIFF)
			prevld[c] = reinterpret_cast<const uint16_t *>(fsrc)[first ? first - 1u : 0u];
		else
			prevld[c] = 0u;
	}
}

template <int PRE, bool STREAM, bool AUTO = false>
__global__ __launch_bounds__(RWG) __attribute__((amdgpu_waves_per_eu(rice_wgpcu<PRE, AUTO>() * RWG / 256u, 8))) void
rice_kernel(KArgs a)
{
	static_assert(!(AUTO && STREAM), "AUTO: frames only");
	// 22-byte header (GOLOMB_ZERO); STREAM (cmp_gpu_encode_stream): one frame,
	// payload only (no header, checksum or 24-bit size field)
	constexpr uint32_t HDR_BITS = STREAM ? 0u : 176u;
	extern __shared__ __attribute__((aligned(16))) uint32_t L_ar[]; // RGUARD words, then the arena
	__shared__ __attribute__((aligned(16))) uint2 s_tab[20];
	// the pair table: entry 18 qa + qb (qa, qb = min(q, 17) of a sample pair)
	// = (P, lb | L << 8): P = (T'[qa] << lb) + T'[qb], lb the second code's
	// length, L the pair's (P meaningless when L > 32)
	__shared__ __attribute__((aligned(16))) uint2 s_ptab[18 * 18];
	__shared__ __attribute__((aligned(16))) uint32_t s_wsum[2][RNW];
	__shared__ uint32_t s_misc[4];

	const uint32_t tid = threadIdx.x, lane = tid & 63u;
	const uint32_t wid = __builtin_amdgcn_readfirstlane(tid >> 6);
	const uint32_t nfr = a.num_segs / a.segs_per_frame;
	// Frame-interleaved order (as encode_kernel): dispatch index d is segment
	// d / nfr of launch frame d % nfr, so a frame's segments come in order.
	// One segment per workgroup, d = the block index.  AUTO: frame-major and
	// XCD-local instead (as encode_kernel's AUTO): frame 8 j + x takes blocks
	// x + 8 (j spf + s), so that a frame's segments, which meet at the
	// candidate barrier, are dispatched together on one XCD; the grid is padded
	// to whole groups of 8 frames.
	const uint32_t d = blockIdx.x;
	uint32_t sif, lf;
	if constexpr (AUTO) {
		const uint32_t p = d >> 3;
		sif = p % a.segs_per_frame;
		lf = 8u * (p / a.segs_per_frame) + (d & 7u);
		if (lf >= nfr)
			return; // padding block
	} else {
		sif = d / nfr;
		lf = d - sif * nfr;
	}
	const uint32_t gseg = lf * a.segs_per_frame + sif;
	const uint32_t frame =
		__builtin_amdgcn_readfirstlane(a.frame_list ? a.frame_list[lf] : a.frame_add + lf * a.frame_mul);
	if (frame == AIRS_NO_FRAME)
		return;
	const uint8_t *const fsrc = a.src + (uint64_t)frame * a.src_stride;
	dbg_stamp(a, gseg, 0);

	// ---- phase 0: every load of the segment, then zero the arena ----------
	uint4 raw[RCH][2];
	uint32_t prevld[RCH];
	rice_load<PRE>(a, fsrc, sif, gseg, tid, raw, prevld);
	if (DBG(262144u)) { // ablation timeline: slot 5 = wave 0's samples landed, 6 = phase 1 done
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		if (wid == 0)
			dbg_stamp(a, gseg, 5);
	}
	{
		// (the arena size is the launch's, a compile-time constant: an unrolled loop)
		constexpr uint32_t IW = rice_arena_words(rice_wgpcu<PRE, AUTO>());
		uint4 *L4 = reinterpret_cast<uint4 *>(L_ar);
#pragma unroll
		for (uint32_t i = 0; i < (IW / 4u + RWG - 1u) / RWG; i++)
			if (i * RWG + tid < IW / 4u)
				L4[i * RWG + tid] = make_uint4(0u, 0u, 0u, 0u);
	}
	const bool is_first = sif == 0u, is_last = sif + 1u == a.segs_per_frame;
	Coder cd;
	uint32_t k, auto_P = 0u;
	uint32_t mp[AUTO ? RCH : 1][8]; // AUTO: the mapped pairs, kept across the frame's k choice
	if constexpr (AUTO) {
		// ---- AUTO: residuals, histogram, the frame's k -----
#pragma unroll
		for (uint32_t c = 0; c < RCH; c++) {
			const uint32_t w[8] = {raw[c][0].x, raw[c][0].y, raw[c][0].z, raw[c][0].w,
					       raw[c][1].x, raw[c][1].y, raw[c][1].z, raw[c][1].w};
			const uint32_t pv0 = (c == 0u && sif == 0u && wid == 0u) ? 0u : prevld[c];
			const uint32_t wprev = PRE == PRE_DIFF ? (uint32_t)__builtin_amdgcn_update_dpp(
									 (int)(pv0 << 16), (int)w[7], 0x138, 0xF, 0xF, false)
							       : 0u;
#pragma unroll
			for (uint32_t j = 0; j < 8u; j++) {
				uint32_t u = w[j];
				if (PRE == PRE_DIFF)
					u = unpk(pk(w[j]) - pk(__builtin_amdgcn_alignbit(w[j], j ? w[j - 1] : wprev, 16)));
				mp[AUTO ? c : 0][j] = zigzag_pk(u);
			}
#pragma unroll
			for (uint32_t j = 0; j < 8u; j++)
				asm volatile("" : "+v"(mp[AUTO ? c : 0][j]));
		}
		const uint2 ks = rice_auto_k(a, L_ar, mp, gseg, sif, tid, lane, wid);
		k = ks.x;
		auto_P = ks.y + HDR_BITS;
		cd = make_coder<ENC_ZERO>(1u << k, a.outlier_param);
		if (tid < 18u)
			s_tab[tid] = rice_table_entry(tid, k);
		rice_pair_table(s_ptab, k, tid);
		__syncthreads(); // the tables; the arena is zero again (rice_auto_k)
	} else {
		cd = make_coder<ENC_ZERO>(__builtin_amdgcn_readfirstlane(a.g), a.outlier_param);
		k = cd.k;
		if (tid < 18u)
			s_tab[tid] = rice_table_entry(tid, k);
		rice_pair_table(s_ptab, k, tid);
		__syncthreads(); // B0: tables and zeroed arena
	}

	// ---- phase 1: codeword pairs and lengths -----------------------------
	// V[c][j]: the codewords of samples 2j, 2j+1 of the lane's chunk c back to
	// back (or the two mapped values when they exceed 32 bits); lp[c]: the
	// eight pair lengths, a byte each; T[c]: their sum
	uint32_t V[RCH][8], lp[RCH][2], T[RCH];
	const char *ptab = reinterpret_cast<const char *>(s_ptab);
#pragma unroll
	for (uint32_t c = 0; c < RCH; c++) {
		const uint32_t w[8] = {raw[c][0].x, raw[c][0].y, raw[c][0].z, raw[c][0].w,
				       raw[c][1].x, raw[c][1].y, raw[c][1].z, raw[c][1].w};
		uint32_t m[8], q8[8]; // q8: min(q, 17) of both samples
		// the pair ending with the sample before the lane's first: lane i - 1's
		// last pair (DPP wave_shr:1), lane 0 the loaded sample
		const uint32_t pv0 = (c == 0u && sif == 0u && wid == 0u) ? 0u : prevld[c]; // 0 before the frame's first sample
		const uint32_t wprev = !AUTO && PRE == PRE_DIFF ? (uint32_t)__builtin_amdgcn_update_dpp(
									  (int)(pv0 << 16), (int)w[7], 0x138, 0xF, 0xF, false)
								: 0u;
#pragma unroll
		for (uint32_t j = 0; j < 8u; j++) {
			if constexpr (AUTO) {
				m[j] = mp[AUTO ? c : 0][j];
			} else {
				uint32_t u = w[j];
				if (PRE == PRE_DIFF)
					u = unpk(pk(w[j]) - pk(__builtin_amdgcn_alignbit(w[j], j ? w[j - 1] : wprev, 16)));
				m[j] = zigzag_pk(u);
			}
			u16x2 q;
			if (!AUTO || k <= 11u) {
				// v = m + 1 saturates at 65535 for m = 65535: the same q after the
				// clamp at 17 while 65535 >> k >= 17, i.e. k <= 11
				const u16x2 v = __builtin_elementwise_add_sat(pk(m[j]), (u16x2)(1));
				q = v >> (u16x2)((unsigned short)k);
			} else {
				// AUTO, k >= 12: (m + 1) >> k = (m >> k) + ((m & (2^k - 1)) + 1) >> k,
				// every term below 2^16
				const u16x2 mk = pk(m[j]);
				const u16x2 lo = (mk & (u16x2)((unsigned short)((1u << k) - 1u))) + (u16x2)(1);
				q = (mk >> (u16x2)((unsigned short)k)) + (lo >> (u16x2)((unsigned short)k));
			}
			q8[j] = unpk(__builtin_elementwise_min(q, (u16x2)(17)));
		}
#pragma unroll
		for (uint32_t h = 0; h < 2u; h++) {
			// one pair-table read per pair: its byte offset 144 qa + 8 qb by
			// one v_dot2 of the packed min(q, 17)
			uint2 te[4];
#pragma unroll
			for (uint32_t jj = 0; jj < 4u; jj++) {
				const uint32_t ofs = __builtin_amdgcn_udot2(pk(q8[4u * h + jj]), (u16x2){144, 8}, 0u, false);
				te[jj] = *reinterpret_cast<const uint2 *>(ptab + ofs);
			}
			uint32_t lw = 0u;
#pragma unroll
			for (uint32_t jj = 0; jj < 4u; jj++) {
				const uint32_t j = 4u * h + jj;
				const uint2 e = te[jj];
				// the codeword pair (m_a << lb) + m_b + P, with the halves of m
				// selected by SDWA
				uint32_t t1, t2, v;
				asm("v_lshlrev_b32_sdwa %0, %2, %3 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
				    "v_add_u32_sdwa %1, %4, %3 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
				    : "=&v"(t1), "=&v"(t2)
				    : "v"(e.y), "v"(m[j]), "v"(e.x));
				uint32_t fast = t1 + t2;
				asm volatile("" : "+v"(fast));
				// pairs of more than 32 bits keep their mapped values: L > 32 is
				// e.y > 0x20FF (l_b < 256), one plain compare (an SDWA compare
				// issues at about half the rate under load, scripts/valu_bench.hip)
				v = e.y > 0x20FFu ? m[j] : fast;
				V[c][j] = v;
				// the length byte into byte jj of lw
				if (jj == 0u)
					asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:BYTE_1" : "=v"(lw) : "v"(e.y));
				else if (jj == 1u)
					asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1" : "+v"(lw) : "v"(e.y));
				else if (jj == 2u)
					asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1" : "+v"(lw) : "v"(e.y));
				else
					asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1" : "+v"(lw) : "v"(e.y));
			}
			lp[c][h] = lw;
		}
		// the chunk's bits: its eight pair lengths (bytes, each <= 64) summed
		// by two v_sad_u8
		T[c] = __builtin_amdgcn_sad_u8(lp[c][0], 0u, __builtin_amdgcn_sad_u8(lp[c][1], 0u, 0u));
		// opaque: keeps the compiler from recomputing the pairs in the packer
#pragma unroll
		for (uint32_t j = 0; j < 8u; j++)
			asm volatile("" : "+v"(V[c][j]));
	}

	if (DBG(262144u) && wid == 0)
		dbg_stamp(a, gseg, 6);
	// ---- block scan of the chunk totals (two chunks per register: a wave's
	// inclusive sums stay below 2^16) --------------------------------------
	const uint32_t inc01 = wave_incl_scan(T[0] | (T[1] << 16));
	const uint32_t inc23 = wave_incl_scan(T[2] | (T[3] << 16));
	if (lane == 63u) {
		s_wsum[0][wid] = inc01;
		s_wsum[1][wid] = inc23;
	}

	// ---- the segment's last 32 bits (wave 3: lanes 60-63, chunk 3) --------
	if (!is_last && wid == RNW - 1) {
		uint64_t acc = 0u;
		const uint2 *tb = s_tab;
#pragma unroll
		for (uint32_t j = 0; j < 8u; j++) {
			const uint32_t L = len_byte(lp[RCH - 1], j);
			if (__ballot(L > 32u) == 0ull) {
				acc = (acc << L) | V[RCH - 1][j];
			} else {
				const bool big = L > 32u;
				const uint2 ca = rice_code(V[RCH - 1][j] & 0xFFFFu, k, tb);
				const uint2 cb = rice_code(V[RCH - 1][j] >> 16, k, tb);
				acc = big ? (acc << ca.y) | ca.x : acc;
				acc = (acc << (big ? cb.y : L)) | (big ? cb.x : V[RCH - 1][j]);
			}
		}
		// (v, t) = the last min(T, 32) bits of a lane run; two scan steps
		// cover four lanes (>= 32 bits: every sample takes >= k + 1 bits)
		uint32_t v = (uint32_t)acc, tbits = min(T[RCH - 1], 32u);
#pragma unroll
		for (uint32_t d = 1; d <= 2; d <<= 1) {
			const uint32_t va = __shfl_up(v, d, 64), ta = __shfl_up(tbits, d, 64);
			if (lane >= d && tbits < 32u) {
				v = (va << tbits) | v;
				tbits = min(ta + tbits, 32u);
			}
		}
		if (lane == 63u)
			gran_store(&a.tail[gseg], ((uint64_t)a.epoch << 32) | v);
	}
	if (DBG(32768u)) { // ablation: stop after phase 1
		if (T[0] == 0x12345u && tid == 999u)
			a.status[0] = V[0][0] + V[RCH - 1][1] + lp[1][1];
		return;
	}
	__syncthreads(); // B1: wave totals

	uint32_t excl[RCH], tot[RCH], base[RCH];
	uint32_t A = 0u;
	{
		uint32_t w01[RNW], w23[RNW];
#pragma unroll
		for (uint32_t w = 0; w < RNW; w += 4) {
			const uint4 s01 = *reinterpret_cast<const uint4 *>(&s_wsum[0][w]);
			const uint4 s23 = *reinterpret_cast<const uint4 *>(&s_wsum[1][w]);
			w01[w] = s01.x, w01[w + 1] = s01.y, w01[w + 2] = s01.z, w01[w + 3] = s01.w;
			w23[w] = s23.x, w23[w + 1] = s23.y, w23[w + 2] = s23.z, w23[w + 3] = s23.w;
		}
		// chunk totals can pass 2^16 across the four waves: carry-free halves
		// of each wave's sum, added in 32 bits
		uint32_t tt[RCH] = {0u, 0u, 0u, 0u}, oo[RCH] = {0u, 0u, 0u, 0u};
#pragma unroll
		for (uint32_t w = 0; w < RNW; w++) {
			tt[0] += w01[w] & 0xFFFFu;
			tt[1] += w01[w] >> 16;
			tt[2] += w23[w] & 0xFFFFu;
			tt[3] += w23[w] >> 16;
			oo[0] += w < wid ? w01[w] & 0xFFFFu : 0u;
			oo[1] += w < wid ? w01[w] >> 16 : 0u;
			oo[2] += w < wid ? w23[w] & 0xFFFFu : 0u;
			oo[3] += w < wid ? w23[w] >> 16 : 0u;
		}
		const uint32_t inc[RCH] = {inc01 & 0xFFFFu, inc01 >> 16, inc23 & 0xFFFFu, inc23 >> 16};
#pragma unroll
		for (uint32_t c = 0; c < RCH; c++) {
			excl[c] = oo[c] + inc[c] - T[c];
			tot[c] = __builtin_amdgcn_readfirstlane(tt[c]);
			base[c] = A;
			A += tot[c];
		}
	}
	if (!AUTO && wid == 0 && lane == 0) { // (AUTO: the offset is known from the candidates)
		const uint64_t tag = ((uint64_t)a.epoch << 1) | (is_first ? 1u : 0u);
		gran_store(&a.agg[gseg], (tag << 32) | (is_first ? HDR_BITS + A : A));
	}
	dbg_stamp(a, gseg, 1);
	uint8_t *fdst = a.dst + (uint64_t)frame * a.dst_stride;
	const uint32_t cap = a.cap;
	const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(fdst, 0, (int)(cap & ~3u), 0x00020000);
	uint32_t *const arena = L_ar + RGUARD;
	const uint32_t abit = (uint32_t)(uintptr_t)arena << 3; // bit address of the arena in LDS
	// the segment fits the arena (with a word to spare for a lane's flush)
	const bool fits = (A >> 5) + 2u <= a.img_words - RGUARD;
	// header bytes 20-21 (low half of the outlier field) share the frame's
	// first payload word
	const uint32_t hdr_pred = STREAM ? 0u : cd.outlier & 0xFFFFu;
	__builtin_amdgcn_s_setprio(1);

	if (fits) {
		// ---- phase 2: the whole segment into the arena, back to back -----
#pragma unroll
		for (uint32_t c = 0; c <= RCH; c++) {
			if (c == AIRS_RICE_LBC && wid == 0) {
				// the look-back (wave 0), once this many chunks are packed
				uint2 pp = make_uint2(HDR_BITS, hdr_pred);
				dbg_stamp(a, gseg, 3);
				if (DBG(2u)) // ablation: no look-back (offsets invented, output garbage)
					pp = make_uint2(HDR_BITS + sif * 37u, 0u);
				else if (AUTO)
					pp = make_uint2(auto_P, is_first ? hdr_pred : rice_tail_wait(a, gseg));
				else if (!is_first)
					pp = (a.lbmode & 1u) && sif >= 16u ? rice_lookback_s(a, gseg, sif, lane)
									     : rice_lookback(a, gseg, sif, lane, 0ull);
				if (lane == 0) {
					if (!AUTO && !is_first)
						gran_store(&a.agg[gseg], ((((uint64_t)a.epoch << 1) | 1u) << 32) | (pp.x + A));
					s_misc[0] = pp.x;
					s_misc[1] = pp.y;
				}
				dbg_stamp(a, gseg, 2);
			}
			if (c < RCH && !(DBG(32u))) { // (ablation 32: no packing)
				RPack p;
				p.init(abit + base[c] + excl[c]);
				pack_chunk(p, V[c], lp[c], k, s_tab);
				p.flush();
			}
		}
		__syncthreads(); // B2: arena complete, offset known
		const uint32_t P = __builtin_amdgcn_readfirstlane(s_misc[0]);
		const uint32_t pred = __builtin_amdgcn_readfirstlane(s_misc[1]);
		if (!(DBG(2048u))) // (ablation 2048: no stores)
			rice_store(arena, P, A, pred, is_last, rsrc, fdst, cap, tid);
		if (is_last && tid == 0)
			s_misc[2] = P;
		dbg_stamp(a, gseg, 4);
	} else {
		// ---- a segment that does not fit: offset first, then chunk by chunk
		// through the arena (every chunk fits: 4096 x (k + 17) bits) --------
		if (wid == 0) {
			uint2 pp = make_uint2(HDR_BITS, hdr_pred);
			if (AUTO)
				pp = make_uint2(auto_P, is_first ? hdr_pred : rice_tail_wait(a, gseg));
			else if (!is_first)
				pp = (a.lbmode & 1u) && sif >= 16u ? rice_lookback_s(a, gseg, sif, lane)
								     : rice_lookback(a, gseg, sif, lane, 0ull);
			if (lane == 0) {
				if (!AUTO && !is_first)
					gran_store(&a.agg[gseg], ((((uint64_t)a.epoch << 1) | 1u) << 32) | (pp.x + A));
				s_misc[0] = pp.x;
				s_misc[1] = pp.y;
			}
		}
		__syncthreads();
		const uint32_t P = __builtin_amdgcn_readfirstlane(s_misc[0]);
		uint32_t pred = __builtin_amdgcn_readfirstlane(s_misc[1]);
		uint32_t last_ne = 0u;
#pragma unroll
		for (uint32_t c = 0; c < RCH; c++)
			last_ne = tot[c] ? c : last_ne;
#pragma unroll
		for (uint32_t c = 0; c < RCH; c++) {
			RPack p;
			p.init(abit + excl[c]);
			pack_chunk(p, V[c], lp[c], k, s_tab);
			p.flush();
			__syncthreads();
			rice_store(arena, P + base[c], tot[c], pred, is_last && c == last_ne, rsrc, fdst, cap, tid);
			// the last 32 bits of this chunk precede the next one
			if (tot[c] >= 32u) {
				const uint32_t s0 = tot[c] - 32u, q = s0 >> 5, sh = s0 & 31u;
				pred = sh ? (arena[q] << sh) | (arena[q + 1] >> (32u - sh)) : arena[q];
			} else if (tot[c]) {
				pred = (pred << tot[c]) | (arena[0] >> (32u - tot[c]));
			}
			__syncthreads();
			for (uint32_t i = tid; i < ((tot[c] + 31u) >> 5) + 1u; i += RWG)
				arena[i] = 0u;
			__syncthreads();
		}
		if (is_last && tid == 0)
			s_misc[2] = P;
	}

	// ---- frame epilogue: checksum, header, status (the frame's last
	// segment; as encode_kernel) ------------------------------------------
	if (STREAM && is_last && tid == 0) {
		const uint32_t payload_bytes = (s_misc[2] + A + 7u) >> 3;
		a.status[frame] = payload_bytes > cap ? ERRV(E_DST_TOO_SMALL) : payload_bytes;
		if (a.needed)
			a.needed[frame] = payload_bytes;
	}
	if (!STREAM && is_last && tid == 0) {
		const uint32_t P = s_misc[2];
		const uint32_t n = a.n;
		const uint32_t payload_bytes = (P + A + 7u) >> 3;
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
			     cd.g, cd.outlier);
		if (((uintptr_t)fdst & 7u) == 0u && cap >= 20u) {
			*reinterpret_cast<uint2 *>(fdst) = make_uint2(bswap32(h[0]), bswap32(h[1]));
			*reinterpret_cast<uint2 *>(fdst + 8) = make_uint2(bswap32(h[2]), bswap32(h[3]));
			*reinterpret_cast<uint32_t *>(fdst + 16) = bswap32(h[4]);
		} else {
#pragma unroll
			for (uint32_t w = 0; w < 5u; w++)
				if (4u * w + 4u <= cap)
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

// The launch, or false when it does not fit this kernel (the caller then
// takes encode_kernel): 16-bit NONE/DIFF GOLOMB_ZERO with one g = 2^k,
// k <= RICE_KMAX, for every frame, no model, whole segments of 16 Ki samples
// (stream: one payload-only frame, n <= AIRS_STREAM_MAX, so its bit offsets,
// at most 24 bits per sample, stay below 2^32).
bool rice_encode(const KArgs &k, uint32_t pre, hipStream_t s, bool stream)
{
	if (pre != PRE_NONE && pre != PRE_DIFF)
		return false;
	if (k.frame_g || k.ktot || k.model_mode || !k.g || (k.g & (k.g - 1u)) || k.g > (1u << RICE_KMAX))
		return false;
	if (k.segs_per_frame == 0u || k.n % RSEGN)
		return false;
	// this kernel's segments (RSEGN samples; the granule arrays hold one per
	// AIRS_SEG-chunk segment of the caller, at least as many)
	KArgs ka = k;
	const uint32_t nfr = k.num_segs / k.segs_per_frame;
	ka.segs_per_frame = k.n / RSEGN;
	ka.num_segs = nfr * ka.segs_per_frame;
	ka.img_words = pre == PRE_DIFF ? rice_arena_words(rice_wgpcu<PRE_DIFF, false>())
				       : rice_arena_words(rice_wgpcu<PRE_NONE, false>());
	// block b runs on XCD b mod 8 (round-robin placement, MI355X_MICROARCH.md):
	// with the frame-interleaved order, segment d and its predecessor d - nfr
	// share an XCD when nfr is a multiple of 8 (speed only: every poll's
	// value is true wherever it runs, and the vector look-back takes over
	// after AIRS_RICE_SPOLL scalar polls)
	ka.lbmode = !stream && nfr % 8u == 0u ? 1u : 0u;
#if AIRS_ABLATE
	static const char *lbm = getenv("AIRS_RICE_LBMODE"); // (ablation builds: the look-back mode)
	if (lbm)
		ka.lbmode = (uint32_t)atoi(lbm);
#endif
	const size_t lds = (size_t)ka.img_words * 4u;
	void (*kern)(KArgs);
	if (stream)
		kern = pre == PRE_DIFF ? rice_kernel<PRE_DIFF, true> : rice_kernel<PRE_NONE, true>;
	else
		kern = pre == PRE_DIFF ? rice_kernel<PRE_DIFF, false> : rice_kernel<PRE_NONE, false>;
	hipLaunchKernelGGL(kern, dim3(ka.num_segs), dim3(RWG), lds, s, ka);
	return true;
}

// CMP_GPU_AUTO_RICE with the k chosen in the kernel (frames of at most
// AUTO_MAX_SPF segments, no model): the Rice kernel with the candidate
// barrier in place of the look-back; false when the launch does not fit it
// (16-bit NONE/DIFF, whole 16 Ki-sample segments, 16-byte aligned frames),
// the caller then takes encode_kernel's AUTO.
bool rice_auto_encode(const KArgs &k, uint32_t pre, hipStream_t s)
{
	if (pre != PRE_NONE && pre != PRE_DIFF)
		return false;
	if (RWG != 256u) // the histogram's row split is for 256 threads
		return false;
	if (!k.ktot || k.frame_g || k.model_mode || k.segs_per_frame == 0u || k.n % RSEGN)
		return false;
	const uint32_t nfr = k.num_segs / k.segs_per_frame;
	KArgs ka = k;
	ka.segs_per_frame = k.n / RSEGN;
	if (ka.segs_per_frame != k.segs_per_frame || ka.segs_per_frame > AUTO_MAX_SPF)
		return false; // (the candidate granules are laid out per caller segment)
	ka.num_segs = nfr * ka.segs_per_frame;
	ka.img_words = pre == PRE_DIFF ? rice_arena_words(rice_wgpcu<PRE_DIFF, true>())
				       : rice_arena_words(rice_wgpcu<PRE_NONE, true>());
	const uint32_t grid = (nfr + 7u) / 8u * 8u * ka.segs_per_frame;
	const size_t lds = (size_t)ka.img_words * 4u;
	if (pre == PRE_DIFF)
		hipLaunchKernelGGL((rice_kernel<PRE_DIFF, false, true>), dim3(grid), dim3(RWG), lds, s, ka);
	else
		hipLaunchKernelGGL((rice_kernel<PRE_NONE, false, true>), dim3(grid), dim3(RWG), lds, s, ka);
	return true;
}

} // namespace airs
