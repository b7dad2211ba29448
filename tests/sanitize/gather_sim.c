/*
 * gather_sim.c -- TEST ONLY.  cmp_gpu_gather (airs-compression_amd/csrc/
 * cmp_gather.c) at WORLD ranks, each rank a thread with its own engine (the
 * host-memory device stub, dev_stub.c) and communicator (fake_rccl.c), under
 * AddressSanitizer + UndefinedBehaviorSanitizer.  One scenario per run: the
 * plain gather (the root's buffer, table and patched identifiers checked
 * against the frames), or a refusal on ONE rank (the root's capacity,
 * alignment or NULL buffer, a peer's NULL frames, an allocation failing on one
 * rank, an error-valued size, a frame that made no draw).  Every rank must
 * return the same value and none may be left waiting: a watchdog ends a run
 * that hangs (exit 3).  Prints "rets r0 r1 ...".
 *   usage: gather_sim WORLD ROOT SCENARIO [LAYOUT]
 */
#include <pthread.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "cmp_gpu.h"
#include "airs_dev.h"

struct fake_shared;
struct ncclComm;
struct fake_shared *fake_shared_new(int world);
struct ncclComm *fake_comm(struct fake_shared *s, int rank);
extern __thread int stub_scratch_fail_slot;

enum {
	S_OK, S_ROOT_SMALL, S_ROOT_MISALIGNED, S_ROOT_OUT_NULL, S_PEER_FRAMES_NULL, S_PEER_FAIL_TABLE,
	S_PEER_FAIL_PACK, S_ROOT_FAIL_TABLE, S_ROOT_FAIL_PATCH, S_ERROR_SIZE, S_NO_DRAW, S_NSCEN
};

#define F 6         /* frames per rank */
#define STRIDE 512u /* frame stride and capacity */

static int W, ROOT, SC, LAYOUT;
static struct fake_shared *SH;
static uint32_t rets[64];
static uint8_t frames_all[64][F * STRIDE];
static uint32_t sizes_all[64][F];

static uint32_t fsize(int r, int j)
{
	return 16u + (uint32_t)((r * 131 + j * 57) % 300);
}

static void *rank_main(void *arg)
{
	const int r = (int)(intptr_t)arg;
	struct cmp_gpu_engine *eng = NULL;
	struct ncclComm *comm = fake_comm(SH, r);
	uint8_t draws[F];
	uint64_t cap = 0, *offs = NULL;
	uint32_t *osz = NULL, e;
	uint8_t *outm = NULL, *out = NULL;
	const void *frames = frames_all[r];
	int j, q;

	if (cmp_gpu_engine_create(&eng, NULL))
		abort();
	for (j = 0; j < F; j++) {
		sizes_all[r][j] = fsize(r, j);
		for (q = 0; q < (int)STRIDE; q++)
			frames_all[r][j * STRIDE + q] = (uint8_t)(r * 37 + j * 11 + q);
		draws[j] = 1;
	}
	if (SC == S_ERROR_SIZE && r == (ROOT + 1) % W)
		sizes_all[r][2] = (uint32_t)0 - 30u;
	if (SC == S_NO_DRAW && r == (ROOT + 1) % W)
		draws[1] = 0;
	if (SC == S_PEER_FRAMES_NULL && r == (ROOT + 1) % W)
		frames = NULL;
	if ((SC == S_PEER_FAIL_TABLE && r == (ROOT + 1) % W) || (SC == S_ROOT_FAIL_TABLE && r == ROOT))
		stub_scratch_fail_slot = AIRS_SLOT_GATHER;
	if (SC == S_PEER_FAIL_PACK && r == (ROOT + 1) % W)
		stub_scratch_fail_slot = AIRS_SLOT_GATHER + 1;
	if (SC == S_ROOT_FAIL_PATCH && r == ROOT)
		stub_scratch_fail_slot = AIRS_SLOT_GATHER + 2;
	if (r == ROOT) {
		int rr;

		for (rr = 0; rr < W; rr++)
			for (j = 0; j < F; j++)
				cap += (fsize(rr, j) + 7u) & ~7u;
		if (SC == S_ROOT_SMALL)
			cap -= 1;
		outm = malloc(cap + 16);
		out = outm + (SC == S_ROOT_MISALIGNED ? 4 : 0);
		if (SC == S_ROOT_OUT_NULL)
			out = NULL;
		offs = calloc((size_t)W * F, 8);
		osz = calloc((size_t)W * F, 4);
	}
	e = cmp_gpu_gather(eng, comm, (uint32_t)ROOT, (uint32_t)LAYOUT, 2u, frames, STRIDE, STRIDE, sizes_all[r], draws,
			   F, out, cap, offs, osz, 1000u, CMP_GPU_GATHER_PATCH_IDS);
	rets[r] = e;
	if (r == ROOT && SC == S_OK && e == 0) {
		/* every frame at its table offset; identifiers 1001, 1002, ... in
		 * global order (one draw per frame, frame layouts) */
		int g, bad = 0;

		for (g = 0; g < W * F; g++) {
			int rr = 0, jj = 0;

			if (LAYOUT == CMP_GPU_LAYOUT_ROUNDROBIN)
				rr = g % W, jj = g / W;
			else if (LAYOUT == CMP_GPU_LAYOUT_BLOCK)
				rr = g / F, jj = g % F;
			else
				rr = (g / 2) % W, jj = (g / 2) / W * 2 + g % 2;
			if (osz[g] != fsize(rr, jj))
				bad = 1;
			for (q = 0; q < (int)osz[g]; q++) {
				uint8_t want = frames_all[rr][jj * STRIDE + q];

				if (q >= 8 && q < 14) {
					/* streams: the identifier of this stream's frames */
					const uint64_t id = LAYOUT == CMP_GPU_LAYOUT_STREAMS ? 1000u + (uint64_t)g + 1u
											     : 1000u + (uint64_t)g + 1u;
					want = (uint8_t)(id >> (8 * (13 - q)));
				}
				if (out[offs[g] + (uint64_t)q] != want)
					bad = 1;
			}
		}
		if (bad)
			rets[r] = 0xBAD;
	}
	free(outm);
	free(offs);
	free(osz);
	cmp_gpu_engine_destroy(eng);
	free(comm);
	return NULL;
}

static void on_alarm(int sig)
{
	(void)sig;
	static const char m[] = "gather_sim: a rank is still waiting (hang)\n";
	(void)!write(2, m, sizeof(m) - 1);
	_exit(3);
}

int main(int argc, char **argv)
{
	pthread_t th[64];
	int r;

	if (argc < 4)
		return 2;
	W = atoi(argv[1]);
	ROOT = atoi(argv[2]);
	SC = atoi(argv[3]);
	LAYOUT = argc > 4 ? atoi(argv[4]) : CMP_GPU_LAYOUT_BLOCK;
	if (W < 1 || W > 64 || ROOT < 0 || SC < 0 || SC >= S_NSCEN)
		return 2;
	SH = fake_shared_new(W);
	signal(SIGALRM, on_alarm);
	alarm(20);
	for (r = 0; r < W; r++)
		pthread_create(&th[r], NULL, rank_main, (void *)(intptr_t)r);
	for (r = 0; r < W; r++)
		pthread_join(th[r], NULL);
	printf("rets");
	for (r = 0; r < W; r++)
		printf(" %u", rets[r]);
	printf("\n");
	return 0;
}
