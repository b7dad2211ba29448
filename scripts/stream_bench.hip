// stream_bench.hip -- the HBM ceiling of cfg2's access pattern on this box:
// 128 MiB of u16 samples read once per launch (cold: three rotated buffers),
// as 4096 segments of 32 KiB, with and without the ~43 % of bytes the encoder
// writes back.  Kernels:
//   seg32    one 256-thread workgroup per segment, lane t reads its 32 B of
//            each 8 KiB chunk (rice_load's pattern: two 16 B loads per lane)
//   coal     one workgroup per segment, each load instruction 1 KiB contiguous
//   pers<G>  G resident workgroups walk the segments (grid stride), the next
//            segment's loads issued before this one is reduced
//   *_w      the same, plus a 14 KiB coalesced store per segment
// Prints one line per kernel: median us over 5 spans of 20 launches, GB/s of
// reads.  Not part of the product (scripts/).
//   hipcc --offload-arch=gfx950 -O3 -o stream_bench scripts/stream_bench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                              \
	do {                                                                               \
		hipError_t e_ = (x);                                                       \
		if (e_ != hipSuccess) {                                                    \
			fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
			exit(1);                                                           \
		}                                                                          \
	} while (0)

constexpr uint32_t SEGB = 32768;           // bytes per segment
constexpr uint32_t NSEG = 4096;            // 128 MiB
constexpr uint32_t WB = 14336;             // bytes written per segment (~0.44)

template <bool W>
__global__ __launch_bounds__(256) void seg32(const uint8_t *src, uint8_t *dst, uint32_t *sink)
{
	const uint32_t t = threadIdx.x;
	const uint8_t *s = src + (uint64_t)blockIdx.x * SEGB;
	uint4 r[8];
#pragma unroll
	for (int c = 0; c < 4; c++) {
		const uint4 *p = reinterpret_cast<const uint4 *>(s + c * 8192 + t * 32);
		r[2 * c] = p[0];
		r[2 * c + 1] = p[1];
	}
	uint32_t x = 0;
#pragma unroll
	for (int i = 0; i < 8; i++)
		x ^= r[i].x + r[i].y * 3u + r[i].z * 5u + r[i].w * 7u;
	if (W) {
		uint4 *d = reinterpret_cast<uint4 *>(dst + (uint64_t)blockIdx.x * SEGB);
		for (uint32_t i = t; i < WB / 16u; i += 256u)
			d[i] = make_uint4(x, x + i, x ^ i, i);
	} else if (x == 0x12345678u)
		sink[blockIdx.x] = x;
}

// writes: MODE 0 strided (segment i at dst + i * 32 KiB), 1 dense (dst + i *
// WB: one contiguous compressed stream, as the encoder writes), 2 dense with
// non-temporal stores; ONLYW: no reads at all
template <int MODE, bool ONLYW>
__global__ __launch_bounds__(256) void segw(const uint8_t *src, uint8_t *dst, uint32_t *sink)
{
	const uint32_t t = threadIdx.x;
	uint32_t x = blockIdx.x;
	if (!ONLYW) {
		const uint8_t *s = src + (uint64_t)blockIdx.x * SEGB;
		uint4 r[8];
#pragma unroll
		for (int c = 0; c < 4; c++) {
			const uint4 *p = reinterpret_cast<const uint4 *>(s + c * 8192 + t * 32);
			r[2 * c] = p[0];
			r[2 * c + 1] = p[1];
		}
#pragma unroll
		for (int i = 0; i < 8; i++)
			x ^= r[i].x + r[i].y * 3u + r[i].z * 5u + r[i].w * 7u;
	}
	uint4 *d = reinterpret_cast<uint4 *>(dst + (uint64_t)blockIdx.x * (MODE == 0 ? SEGB : WB));
	for (uint32_t i = t; i < WB / 16u; i += 256u) {
		const uint4 v = make_uint4(x, x + i, x ^ i, i);
		if (MODE == 2) {
			typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
			u32x4 w = {v.x, v.y, v.z, v.w};
			__builtin_nontemporal_store(w, reinterpret_cast<u32x4 *>(d + i));
		} else {
			d[i] = v;
		}
	}
	if (x == 0x12345678u)
		sink[blockIdx.x] = x;
}

template <bool W>
__global__ __launch_bounds__(256) void coal(const uint8_t *src, uint8_t *dst, uint32_t *sink)
{
	const uint32_t t = threadIdx.x;
	const uint4 *p = reinterpret_cast<const uint4 *>(src + (uint64_t)blockIdx.x * SEGB);
	uint4 r[8];
#pragma unroll
	for (int i = 0; i < 8; i++)
		r[i] = p[i * 256 + t];
	uint32_t x = 0;
#pragma unroll
	for (int i = 0; i < 8; i++)
		x ^= r[i].x + r[i].y * 3u + r[i].z * 5u + r[i].w * 7u;
	if (W) {
		uint4 *d = reinterpret_cast<uint4 *>(dst + (uint64_t)blockIdx.x * SEGB);
		for (uint32_t i = t; i < WB / 16u; i += 256u)
			d[i] = make_uint4(x, x + i, x ^ i, i);
	} else if (x == 0x12345678u)
		sink[blockIdx.x] = x;
}

// persistent: segment b, b + G, ...; the next segment's loads are issued
// before this one's values are used
template <bool W>
__global__ __launch_bounds__(256) void pers(const uint8_t *src, uint8_t *dst, uint32_t *sink)
{
	const uint32_t t = threadIdx.x, G = gridDim.x;
	uint4 r[8], nx[8];
	uint32_t seg = blockIdx.x;
	{
		const uint4 *p = reinterpret_cast<const uint4 *>(src + (uint64_t)seg * SEGB);
#pragma unroll
		for (int i = 0; i < 8; i++)
			r[i] = p[i * 256 + t];
	}
	uint32_t acc = 0;
	for (; seg < NSEG; seg += G) {
		const uint32_t nseg = seg + G < NSEG ? seg + G : seg;
		const uint4 *p = reinterpret_cast<const uint4 *>(src + (uint64_t)nseg * SEGB);
#pragma unroll
		for (int i = 0; i < 8; i++)
			nx[i] = p[i * 256 + t];
		uint32_t x = 0;
#pragma unroll
		for (int i = 0; i < 8; i++)
			x ^= r[i].x + r[i].y * 3u + r[i].z * 5u + r[i].w * 7u;
		if (W) {
			uint4 *d = reinterpret_cast<uint4 *>(dst + (uint64_t)seg * SEGB);
			for (uint32_t i = t; i < WB / 16u; i += 256u)
				d[i] = make_uint4(x, x + i, x ^ i, i);
		}
		acc += x;
#pragma unroll
		for (int i = 0; i < 8; i++)
			r[i] = nx[i];
	}
	if (acc == 0x12345678u)
		sink[blockIdx.x] = acc;
}

typedef void (*kfn)(const uint8_t *, uint8_t *, uint32_t *);

int main()
{
	const size_t bytes = (size_t)SEGB * NSEG;
	const int ROT = 3;
	std::vector<uint8_t *> src(ROT), dst(ROT);
	uint32_t *sink;
	for (int i = 0; i < ROT; i++) {
		CK(hipMalloc(&src[i], bytes));
		CK(hipMalloc(&dst[i], bytes));
		CK(hipMemset(src[i], i + 1, bytes));
		CK(hipMemset(dst[i], 0, bytes));
	}
	CK(hipMalloc(&sink, NSEG * 4));
	struct K {
		const char *name;
		kfn f;
		uint32_t grid;
	} ks[] = {
		{"seg32", seg32<false>, NSEG},   {"seg32_w", seg32<true>, NSEG}, {"coal", coal<false>, NSEG},
		{"coal_w", coal<true>, NSEG},    {"pers1024", pers<false>, 1024}, {"pers1024_w", pers<true>, 1024},
		{"pers2048", pers<false>, 2048}, {"pers2048_w", pers<true>, 2048}, {"pers512_w", pers<true>, 512},
		{"w_strided", segw<0, false>, NSEG}, {"w_dense", segw<1, false>, NSEG}, {"w_dense_nt", segw<2, false>, NSEG},
		{"wonly_dense", segw<1, true>, NSEG}, {"wonly_nt", segw<2, true>, NSEG},
	};
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	for (int rep = 0; rep < 2; rep++)
		for (auto &k : ks) {
			for (int i = 0; i < 10; i++)
				hipLaunchKernelGGL(k.f, dim3(k.grid), dim3(256), 0, 0, src[i % ROT], dst[i % ROT], sink);
			std::vector<float> ms;
			for (int s = 0; s < 5; s++) {
				CK(hipEventRecord(e0, 0));
				for (int i = 0; i < 20; i++)
					hipLaunchKernelGGL(k.f, dim3(k.grid), dim3(256), 0, 0, src[i % ROT], dst[i % ROT], sink);
				CK(hipEventRecord(e1, 0));
				CK(hipEventSynchronize(e1));
				float m;
				CK(hipEventElapsedTime(&m, e0, e1));
				ms.push_back(m / 20.0f);
			}
			std::sort(ms.begin(), ms.end());
			const double us = ms[2] * 1e3;
			printf("%-12s %7.2f us  %7.1f GB/s read%s\n", k.name, us, bytes / (us * 1e-6) / 1e9,
			       rep == 0 ? "  (first pass)" : "");
		}
	return 0;
}
