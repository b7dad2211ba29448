/*
 * fake_rccl.c -- TEST ONLY.  The eight RCCL entry points cmp_gather.c uses,
 * for ranks that are threads of one process over host memory (the device
 * layer is tests/sanitize/dev_stub.c), so that cmp_gpu_gather's multi-rank
 * protocol runs on the CPU: gather_sim.c links it with -rdynamic and
 * cmp_gather.c finds these symbols before it would dlopen librccl.  A rank
 * that never enters a collective its peers entered leaves them waiting here,
 * as it would in RCCL: the harness's watchdog turns that into a failure.
 * Never linked into the product.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include <rccl/rccl.h>

#define FMAX 64

struct fake_shared {
	int world;
	pthread_mutex_t mu;
	pthread_cond_t cv;
	/* all-gather: generation counter and arrivals */
	unsigned ag_gen, ag_in, ag_out;
	const void *ag_src[FMAX];
	size_t ag_len;
	/* point-to-point: a posted send from -> to */
	const void *sbuf[FMAX][FMAX];
	size_t slen[FMAX][FMAX];
	int posted[FMAX][FMAX], taken[FMAX][FMAX];
};

struct ncclComm {
	int rank;
	struct fake_shared *s;
};

struct fake_op {
	int send, peer;
	void *buf;
	size_t len;
	struct ncclComm *c;
};
static __thread int g_depth;
static __thread int g_nop;
static __thread struct fake_op g_op[FMAX * 2];

struct fake_shared *fake_shared_new(int world)
{
	struct fake_shared *s = calloc(1, sizeof(*s));

	s->world = world;
	pthread_mutex_init(&s->mu, NULL);
	pthread_cond_init(&s->cv, NULL);
	return s;
}

struct ncclComm *fake_comm(struct fake_shared *s, int rank)
{
	struct ncclComm *c = calloc(1, sizeof(*c));

	c->rank = rank;
	c->s = s;
	return c;
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int *count)
{
	*count = comm->s->world;
	return ncclSuccess;
}

ncclResult_t ncclCommUserRank(const ncclComm_t comm, int *rank)
{
	*rank = comm->rank;
	return ncclSuccess;
}

const char *ncclGetErrorString(ncclResult_t r)
{
	return r == ncclSuccess ? "success" : "fake rccl error";
}

static size_t tsize(ncclDataType_t t)
{
	return t == ncclUint8 || t == ncclInt8 ? 1u : t == ncclFloat64 || t == ncclUint64 || t == ncclInt64 ? 8u : 4u;
}

ncclResult_t ncclAllGather(const void *sendbuff, void *recvbuff, size_t count, ncclDataType_t type, ncclComm_t comm,
			   hipStream_t stream)
{
	struct fake_shared *s = comm->s;
	const size_t len = count * tsize(type);
	unsigned gen;
	int r;

	(void)stream;
	pthread_mutex_lock(&s->mu);
	while (s->ag_out) /* the previous all-gather is still being read */
		pthread_cond_wait(&s->cv, &s->mu);
	gen = s->ag_gen;
	s->ag_src[comm->rank] = sendbuff;
	s->ag_len = len;
	if (++s->ag_in == (unsigned)s->world) {
		s->ag_in = 0;
		s->ag_out = (unsigned)s->world;
		s->ag_gen++;
		pthread_cond_broadcast(&s->cv);
	}
	while (s->ag_gen == gen)
		pthread_cond_wait(&s->cv, &s->mu);
	for (r = 0; r < s->world; r++)
		memcpy((char *)recvbuff + (size_t)r * len, s->ag_src[r], len);
	if (--s->ag_out == 0)
		pthread_cond_broadcast(&s->cv);
	/* every rank has read every send buffer before any returns (a caller may
	 * free its send buffer once the call is complete) */
	while (s->ag_out && s->ag_gen == gen + 1u)
		pthread_cond_wait(&s->cv, &s->mu);
	pthread_mutex_unlock(&s->mu);
	return ncclSuccess;
}

ncclResult_t ncclGroupStart(void)
{
	g_depth++;
	return ncclSuccess;
}

static ncclResult_t run_ops(void)
{
	int i;

	/* post every send, then serve every receive, then wait for the sends */
	for (i = 0; i < g_nop; i++)
		if (g_op[i].send) {
			struct fake_shared *s = g_op[i].c->s;
			const int me = g_op[i].c->rank, p = g_op[i].peer;

			pthread_mutex_lock(&s->mu);
			s->sbuf[me][p] = g_op[i].buf;
			s->slen[me][p] = g_op[i].len;
			s->taken[me][p] = 0;
			s->posted[me][p] = 1;
			pthread_cond_broadcast(&s->cv);
			pthread_mutex_unlock(&s->mu);
		}
	for (i = 0; i < g_nop; i++)
		if (!g_op[i].send) {
			struct fake_shared *s = g_op[i].c->s;
			const int me = g_op[i].c->rank, p = g_op[i].peer;

			pthread_mutex_lock(&s->mu);
			while (!s->posted[p][me])
				pthread_cond_wait(&s->cv, &s->mu);
			if (s->slen[p][me] != g_op[i].len)
				abort(); /* mismatched transfer sizes: a protocol bug */
			memcpy(g_op[i].buf, s->sbuf[p][me], g_op[i].len);
			s->posted[p][me] = 0;
			s->taken[p][me] = 1;
			pthread_cond_broadcast(&s->cv);
			pthread_mutex_unlock(&s->mu);
		}
	for (i = 0; i < g_nop; i++)
		if (g_op[i].send) {
			struct fake_shared *s = g_op[i].c->s;
			const int me = g_op[i].c->rank, p = g_op[i].peer;

			pthread_mutex_lock(&s->mu);
			while (!s->taken[me][p])
				pthread_cond_wait(&s->cv, &s->mu);
			s->taken[me][p] = 0;
			pthread_mutex_unlock(&s->mu);
		}
	g_nop = 0;
	return ncclSuccess;
}

ncclResult_t ncclGroupEnd(void)
{
	if (g_depth <= 0)
		return ncclInvalidUsage;
	if (--g_depth)
		return ncclSuccess;
	return run_ops();
}

static ncclResult_t add_op(int send, const void *buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm)
{
	if (g_nop >= FMAX * 2 || peer < 0 || peer >= comm->s->world)
		return ncclInvalidArgument;
	g_op[g_nop].send = send;
	g_op[g_nop].peer = peer;
	g_op[g_nop].buf = (void *)buf;
	g_op[g_nop].len = count * tsize(type);
	g_op[g_nop].c = comm;
	g_nop++;
	return g_depth ? ncclSuccess : run_ops();
}

ncclResult_t ncclSend(const void *sendbuff, size_t count, ncclDataType_t type, int peer, ncclComm_t comm,
		      hipStream_t stream)
{
	(void)stream;
	return add_op(1, sendbuff, count, type, peer, comm);
}

ncclResult_t ncclRecv(void *recvbuff, size_t count, ncclDataType_t type, int peer, ncclComm_t comm,
		      hipStream_t stream)
{
	(void)stream;
	return add_op(0, recvbuff, count, type, peer, comm);
}
