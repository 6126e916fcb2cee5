/*
 * gpucsum_module.c -- the io_module_func decorator of gpucsum_io_module.h.
 *
 * Semantics follow the reference's checksum-offload contract:
 *   dev_ioctl answers      dpdk_module.c:805-928 (0 = device did it, -1 = software)
 *   bad-checksum RX drop   dpdk_get_rptr returning NULL, dpdk_module.c:536-542,
 *                          counted by core.c:794-799 as rx_errors
 *   TX ownership           a get_wptr buffer is complete once the next get_wptr /
 *                          send_pkts is called (mTCP writes each frame fully in
 *                          SendTCPPacket before asking for the next, tcp_out.c:223-357)
 *   RX ownership           get_rptr pointers live until the next recv_pkts on the
 *                          same ifidx (dpdk_module.c:458-461)
 * The checksum work itself is libmtcp_gpucsum's gcs_verify_ptrs /
 * gcs_compute_ptrs (one GPU batch per burst).  There is no CPU fallback: a
 * context that cannot reach its GPU exits at init_handle like the reference's
 * modules do (dpdk_module.c:243-247).  A failing call later is counted and
 * reported on stderr, and its frames follow gpucsum_io_module.h's "GPU
 * failures": RX frames come back NULL; TX frames of an in-place inner go out
 * with the check fields mTCP left at 0 (counted: tx_unfilled_sent), shadow
 * (TX_EAGER) frames are withheld; GPUCSUM_ON_GPU_FAIL=exit makes it fatal.
 *
 * Inner-module shapes (gpucsum_io_module.h): frames are filled in place for
 * modules whose TX buffers stay put until send_pkts (dpdk, onvm, psio), and
 * through shadow slots for modules whose get_wptr transmits (netmap).
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/mtcp_gpucsum.h"
#include "../../include/gpucsum_io_module.h"

#define GPUCSUM_MAX_THREADS 256
#define GPUCSUM_STAGE_BYTES_PER_FRAME 2048   /* MAX_PKT_SIZE, mtcp.h:52 */
#define GPUCSUM_SHADOW_ROOM 2048             /* MAX_PKT_SIZE: mTCP never asks for more */
#define GPUCSUM_DEFAULT_SEG_MAX 1514         /* ETHERNET_HEADER_LEN + 1500 B MTU */
#define V_INNER 0xFE                         /* RX_CHAINED frame: inner's own checks */
#define GPUCSUM_ASYNC_MAX 512                /* frames per async post (gcs_compute_ptrs_async) */

struct rx_if {
	int32_t n;
	uint32_t cap;
	uint8_t **ptr;
	uint16_t *len;      /* length seen at recv_pkts            */
	uint16_t *glen;     /* length the GPU folds (0 = skip)      */
	uint8_t *verdict;
	uint16_t *queue;    /* RSS on */
	/* verify as you go (GPUCSUM_RX_GROUP): the burst is posted in groups of
	 * rx_group frames; frames [0, ready) have their verdicts */
	uint32_t ready;
	uint32_t ngroups;
	uint64_t *ticket;   /* per group (0: verified synchronously) */
};

struct tx_if {
	uint32_t n;
	uint32_t done;      /* frames [0, done) are complete (mTCP moved on from them) */
	uint32_t posted;    /* frames [0, posted) are posted to the GPU (async fill)  */
	uint64_t ticket;    /* the last async post's ticket (0: none)                */
	uint8_t *ptr[GPUCSUM_MAX_BURST];
	uint16_t len[GPUCSUM_MAX_BURST];
	uint8_t status[GPUCSUM_MAX_BURST];
	uint8_t *shadow;    /* TX_EAGER: GPUCSUM_MAX_BURST rooms of GPUCSUM_SHADOW_ROOM */
};

struct gthr {
	struct mtcp_thread_context *ctx;
	gcs_ctx *gcs;
	uint32_t tx_group;      /* async TX fill: post every tx_group completed frames (0: off) */
	uint32_t rx_group;      /* async RX verify: frames per posted group (0: one sync batch) */
	struct rx_if *rx[GPUCSUM_MAX_IFS];
	struct tx_if *tx[GPUCSUM_MAX_IFS];
	struct tx_if *last_tx;  /* the queue of the most recent get_wptr */
	struct gpucsum_stats st;
	int rss;                /* RSS steering check on */
	int own_queue;
};

/* mTCP's netmap module, when the decorator is linked into mTCP (weak: absent
 * from other programs).  Its get_wptr transmits, netmap_module.c:149-160. */
extern io_module_func netmap_module_func __attribute__((weak));
/* ... and its DPDK module.  Without ENABLELRO it receives no frame longer than
 * 1518 B (jumbo frames off, max_rx_pkt_len = ETHER_MAX_LEN, dpdk_module.c:
 * 112-135), so any longer frame is an LRO chain (BUF_SIZE 16384, :44-48)
 * and RX_CHAINED is safe to assume for it either way. */
extern io_module_func dpdk_module_func __attribute__((weak));
/* ... defined by the integration patch in a DPDK module built with IP_DEFRAG,
 * whose get_rptr feeds the reassembly table on every call (dpdk_module.c:
 * 474-513, 527-529): then the inner get_rptr is called once per index. */
extern const int dpdk_module_ip_defrag __attribute__((weak));

static io_module_func *g_inner;
static uint32_t g_caps;
static int g_fail_exit;      /* GPUCSUM_ON_GPU_FAIL=exit: a failed GPU call is fatal */
static uint32_t g_seg_max = GPUCSUM_DEFAULT_SEG_MAX;
static struct gthr *g_table[GPUCSUM_MAX_THREADS];
static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;
static int g_next_ordinal;
static __thread struct gthr *t_cache;

int gpucsum_set_inner(io_module_func *inner)
{
	if (!inner || inner == &gpucsum_module_func)
		return GCS_EINVAL;
	g_inner = inner;
	g_caps = 0;
	if (&netmap_module_func && inner == &netmap_module_func)
		g_caps = GPUCSUM_INNER_TX_EAGER;
	if (&dpdk_module_func && inner == &dpdk_module_func)
		g_caps = (&dpdk_module_ip_defrag && dpdk_module_ip_defrag) ? GPUCSUM_INNER_RX_ONCE
		                                                           : GPUCSUM_INNER_RX_CHAINED;
	g_seg_max = GPUCSUM_DEFAULT_SEG_MAX;
	return GCS_OK;
}

io_module_func *gpucsum_get_inner(void)
{
	return g_inner;
}

int gpucsum_set_inner_caps(uint32_t caps, uint32_t rx_seg_max)
{
	const uint32_t known = GPUCSUM_INNER_TX_EAGER | GPUCSUM_INNER_RX_CHAINED |
	                       GPUCSUM_INNER_RX_ONCE;

	if (!g_inner || (caps & ~known) || rx_seg_max > 65535 ||
	    ((caps & GPUCSUM_INNER_RX_ONCE) && (caps & GPUCSUM_INNER_RX_CHAINED)))
		return GCS_EINVAL;
	g_caps = caps;
	g_seg_max = rx_seg_max ? rx_seg_max : GPUCSUM_DEFAULT_SEG_MAX;
	return GCS_OK;
}

uint32_t gpucsum_get_inner_caps(void)
{
	return g_caps;
}

static struct gthr *lookup(struct mtcp_thread_context *ctx)
{
	struct gthr *g = t_cache;
	int i;

	if (g && g->ctx == ctx)
		return g;
	g = NULL;
	pthread_mutex_lock(&g_lock);
	for (i = 0; i < GPUCSUM_MAX_THREADS; i++)
		if (g_table[i] && g_table[i]->ctx == ctx) {
			g = g_table[i];
			break;
		}
	pthread_mutex_unlock(&g_lock);
	if (g)
		t_cache = g;
	return g;
}

static void die(const char *what, int rc)
{
	fprintf(stderr, "[gpucsum] %s failed: %s (%d) %s\n", what, gcs_strerror(rc), rc,
	        gcs_last_hip_error());
	exit(EXIT_FAILURE);
}

/* A GPU call failed after init: count it, report it (the first few and then
 * every 1024th, so a dead GPU does not flood stderr), or exit when
 * GPUCSUM_ON_GPU_FAIL=exit. */
static void gpu_failed(struct gthr *g, const char *what, uint32_t frames, int rc)
{
	g->st.gpu_failures++;
	if (g_fail_exit)
		die(what, rc);
	if (g->st.gpu_failures <= 8 || (g->st.gpu_failures & 1023) == 0)
		fprintf(stderr, "[gpucsum] %s of %u frames failed (failure %llu): %s %s\n", what,
		        frames, (unsigned long long)g->st.gpu_failures, gcs_strerror(rc),
		        gcs_last_hip_error());
}

/* ---- vtable ------------------------------------------------------------ */

static void gpucsum_load_module(void)
{
	int n = 0, rc;

	if (!g_inner) {
		fprintf(stderr, "[gpucsum] no inner I/O module: call gpucsum_set_inner() first\n");
		exit(EXIT_FAILURE);
	}
	/* HIP's default hardware queues suffice: the threads of one GPU share
	 * one resident burst grid, on a stream of its own (gcs_api.cpp
	 * ServerHub; 12 threads per GPU: 23 us per burst with 4 queues, 22 us
	 * with 16, tools/mt_probe.py) */
	rc = gcs_device_count(&n);
	if (rc || n <= 0)
		die("gcs_device_count (no MI355X visible)", rc ? rc : GCS_ENODEV);
	{
		const char *f = getenv("GPUCSUM_ON_GPU_FAIL");
		g_fail_exit = f && strcmp(f, "exit") == 0;
	}
	if (g_inner->load_module)
		g_inner->load_module();
}

static void gpucsum_init_handle(struct mtcp_thread_context *ctx)
{
	struct gthr *g;
	int ndev = 0, dev, ordinal, i, rc;
	const char *env = getenv("GPUCSUM_DEVICE");

	if (g_inner->init_handle)
		g_inner->init_handle(ctx);
	g = calloc(1, sizeof(*g));
	if (!g)
		die("calloc", GCS_ENOMEM);
	g->ctx = ctx;
	pthread_mutex_lock(&g_lock);
	ordinal = g_next_ordinal++;
	for (i = 0; i < GPUCSUM_MAX_THREADS && g_table[i]; i++)
		;
	if (i == GPUCSUM_MAX_THREADS) {
		pthread_mutex_unlock(&g_lock);
		die("thread table", GCS_ERANGE);
	}
	g_table[i] = g;
	pthread_mutex_unlock(&g_lock);

	rc = gcs_device_count(&ndev);
	if (rc || ndev <= 0)
		die("gcs_device_count", rc ? rc : GCS_ENODEV);
	dev = env ? atoi(env) : ordinal % ndev;   /* mTCP thread k -> GPU k mod n */
	rc = gcs_ctx_create(&g->gcs, dev, GPUCSUM_MAX_BURST,
	                    (uint64_t)GPUCSUM_MAX_BURST * GPUCSUM_STAGE_BYTES_PER_FRAME);
	if (rc)
		die("gcs_ctx_create", rc);
	g->st.device = dev;
	t_cache = g;
	/* bursts go to the resident burst grid unless GPUCSUM_BURST_SERVER=0
	 * (64 x 1500 B: ~9 us per burst instead of ~19 us with a launch each) */
	env = getenv("GPUCSUM_BURST_SERVER");
	if (!env || atoi(env) != 0) {
		rc = gcs_ctx_set_burst_server(g->gcs, 1);
		if (rc && rc != GCS_ERANGE)
			die("gcs_ctx_set_burst_server", rc);
		/* GCS_ERANGE: 32 threads of this process already share the
		 * device's grid; this one launches per burst */
		/* fill as you go: a TX frame is complete once mTCP asks for the next
		 * one or for its checksum (tcp_out.c:239-333); every
		 * GPUCSUM_TX_GROUP (default 16, 0 = off) completed frames go to the
		 * server while mTCP builds the rest, so send_pkts waits only for
		 * the last group (round 4, tools/tx_async_probe.py: send_pkts blocks
		 * 6.6 / 6.2 us registered / pageable with 16, 8.7 / 5.8 with 8, 8.5 /
		 * 9.1 with one batch) */
		env = getenv("GPUCSUM_TX_GROUP");
		g->tx_group = rc ? 0 : env ? (uint32_t)atoi(env) : 16;
		/* verify as you go (GPUCSUM_RX_GROUP > 0): recv_pkts posts the burst
		 * in groups of that many frames and returns; get_rptr(i) waits only
		 * for the group holding frame i, so mTCP processes the first frames
		 * (core.c:792-795) while the GPU verifies the rest.  Default 0, one
		 * batch per burst: under the reference's RX loop it blocks 9.5 us
		 * per 64 x 1500 B burst in a registered pool against 11.5 us in
		 * groups of 16 (pageable: 13.9 vs 13.0; tools/rx_async_probe.py) --
		 * every group past the first costs its serving blocks one more poll */
		env = getenv("GPUCSUM_RX_GROUP");
		g->rx_group = rc ? 0 : env ? (uint32_t)atoi(env) : 0;
	}
	env = getenv("GPUCSUM_RSS_QUEUES");
	if (env && atoi(env) > 0) {
		const char *e40 = getenv("GPUCSUM_RSS_I40E");
		rc = gpucsum_set_rss(ctx, NULL, 0, (uint32_t)atoi(env), e40 && atoi(e40),
		                     ordinal % atoi(env));
		if (rc)
			die("gpucsum_set_rss", rc);
	}
}

static int32_t gpucsum_link_devices(struct mtcp_thread_context *ctx)
{
	return g_inner->link_devices ? g_inner->link_devices(ctx) : 0;
}

static void gpucsum_release_pkt(struct mtcp_thread_context *ctx, int ifidx,
                                unsigned char *pkt_data, int len)
{
	if (g_inner->release_pkt)
		g_inner->release_pkt(ctx, ifidx, pkt_data, len);
}

static struct tx_if *txq(struct gthr *g, int ifidx)
{
	struct tx_if *q;

	if (ifidx < 0 || ifidx >= GPUCSUM_MAX_IFS)
		return NULL;
	if (g->tx[ifidx])
		return g->tx[ifidx];
	q = calloc(1, sizeof(struct tx_if));
	if (q && (g_caps & GPUCSUM_INNER_TX_EAGER)) {
		q->shadow = malloc((size_t)GPUCSUM_MAX_BURST * GPUCSUM_SHADOW_ROOM);
		if (!q->shadow) {
			free(q);
			q = NULL;
		}
	}
	g->tx[ifidx] = q;
	return q;
}

/* Async fill of the completed frames not yet posted: [posted, done). */
static void post_tx(struct gthr *g, struct tx_if *q)
{
	uint64_t t = 0;
	int rc;

	if (q->done <= q->posted)
		return;
	rc = gcs_compute_ptrs_async(g->gcs, q->ptr + q->posted, q->len + q->posted,
	                            q->done - q->posted, q->status + q->posted, NULL, &t);
	if (rc) {
		/* leave them to flush_tx's synchronous fill; no more async posts on
		 * this context */
		gpu_failed(g, "async TX fill post", q->done - q->posted, rc);
		g->tx_group = 0;
		return;
	}
	if (t)
		q->ticket = t;
	g->st.tx_posts++;
	q->posted = q->done;
}

/* Frames [0, upto) of queue q are complete: post them once a group is ready. */
static void tx_complete(struct gthr *g, struct tx_if *q, uint32_t upto)
{
	if (upto > q->done)
		q->done = upto;
	if (g->tx_group && q->done - q->posted >= g->tx_group)
		post_tx(g, q);
}

/* TX fill of every queued frame of one interface (ip_out.c:155-173 and
 * tcp_out.c:323-333, batched).  TX_EAGER: the queued frames are shadow slots;
 * once filled they go, in order, into inner get_wptr buffers (the inner may
 * transmit the previous one on each call, netmap_module.c:155-156).  With the
 * async fill, earlier groups are in flight already: post the tail, wait. */
static void flush_tx(struct gthr *g, int ifidx, struct tx_if *q)
{
	uint32_t k, unfilled = 0;
	int rc = 0;

	if (!q || q->n == 0)
		return;
	if (q->posted > 0 || (g->tx_group && q->n <= GPUCSUM_ASYNC_MAX)) {
		q->done = q->n;
		post_tx(g, q);
		if (q->ticket) {
			/* a failed wait cancels every posted fill (gcs_wait) */
			rc = gcs_wait(g->gcs, q->ticket);
			if (rc) {
				unfilled += q->posted;
				gpu_failed(g, "TX fill (async wait)", q->posted, rc);
			}
		}
		if (q->posted < q->n) {
			/* the tail could not be posted: fill it synchronously */
			int rc2 = gcs_compute_ptrs(g->gcs, q->ptr + q->posted, q->len + q->posted,
			                           q->n - q->posted, q->status + q->posted, NULL);
			if (rc2) {
				unfilled += q->n - q->posted;
				gpu_failed(g, "TX fill", q->n - q->posted, rc2);
				rc = rc2;
			}
		}
	} else {
		rc = gcs_compute_ptrs(g->gcs, q->ptr, q->len, q->n, q->status, NULL);
		if (rc) {
			unfilled = q->n;
			gpu_failed(g, "TX fill", q->n, rc);
		}
	}
	q->done = q->posted = 0;
	q->ticket = 0;
	if (!rc) {
		g->st.tx_frames += q->n;
		g->st.tx_batches++;
	}
	if (q->shadow) {
		if (rc) {
			/* unfilled frames never reach the wire: the whole flush is
			 * withheld, so what goes out stays in mTCP's order */
			g->st.tx_unfilled_dropped += q->n;
		} else {
			for (k = 0; k < q->n; k++) {
				uint8_t *p = g_inner->get_wptr(g->ctx, ifidx, q->len[k]);
				if (!p) {
					g->st.tx_inner_full += q->n - k;
					break;
				}
				memcpy(p, q->ptr[k], q->len[k]);
			}
		}
	} else {
		/* in place: the inner sends them as they are (check fields 0) */
		g->st.tx_unfilled_sent += unfilled;
	}
	q->n = 0;
}

static uint8_t *gpucsum_get_wptr(struct mtcp_thread_context *ctx, int ifidx, uint16_t len)
{
	struct gthr *g = lookup(ctx);
	struct tx_if *q;
	uint8_t *p;

	if (!g)
		return g_inner->get_wptr(ctx, ifidx, len);
	q = txq(g, ifidx);
	if (!q)   /* no queue: nothing would fill this frame, so give no buffer */
		return NULL;
	if (q->n == GPUCSUM_MAX_BURST)
		flush_tx(g, ifidx, q);  /* all queued frames are complete by now */
	else
		tx_complete(g, q, q->n);   /* the frames handed out so far are complete */
	if (q->shadow) {
		if (len > GPUCSUM_SHADOW_ROOM)
			return NULL;
		p = q->shadow + (size_t)q->n * GPUCSUM_SHADOW_ROOM;
	} else {
		p = g_inner->get_wptr(ctx, ifidx, len);
		if (!p)
			return NULL;
	}
	q->ptr[q->n] = p;
	q->len[q->n] = len;
	q->n++;
	g->last_tx = q;
	return p;
}

static int32_t gpucsum_send_pkts(struct mtcp_thread_context *ctx, int nif)
{
	struct gthr *g = lookup(ctx);

	if (g && nif >= 0 && nif < GPUCSUM_MAX_IFS)
		flush_tx(g, nif, g->tx[nif]);
	return g_inner->send_pkts(ctx, nif);
}

/* Room for a burst of n frames (an inner module may return more than
 * GPUCSUM_MAX_BURST at once; gcs_*_ptrs splits a batch by itself). */
static int rx_reserve(struct rx_if *r, uint32_t n)
{
	uint32_t cap = r->cap ? r->cap : 64;
	void *a, *b, *c, *d, *e, *f;

	if (n <= r->cap)
		return 0;
	while (cap < n)
		cap *= 2;
	a = realloc(r->ptr, cap * sizeof(*r->ptr));
	if (a) r->ptr = a;
	b = realloc(r->len, cap * sizeof(*r->len));
	if (b) r->len = b;
	c = realloc(r->glen, cap * sizeof(*r->glen));
	if (c) r->glen = c;
	d = realloc(r->verdict, cap);
	if (d) r->verdict = d;
	e = realloc(r->queue, cap * sizeof(*r->queue));
	if (e) r->queue = e;
	f = realloc(r->ticket, cap * sizeof(*r->ticket));   /* >= groups of any size */
	if (f) r->ticket = f;
	if (!a || !b || !c || !d || !e || !f)
		return -1;
	r->cap = cap;
	return 0;
}

/* Frames [lo, hi) have their GPU verdicts: apply the decorator's own
 * dispositions (inner drops, chains left to the inner's checks) and the RSS
 * bookkeeping. */
static void rx_settle(struct gthr *g, struct rx_if *r, int32_t lo, int32_t hi, int rss_ok)
{
	int32_t i;

	for (i = lo; i < hi; i++) {
		if (!r->ptr[i])
			r->verdict[i] = GCS_V_DROP_TRUNC;   /* the inner module's own drop */
		else if (r->glen[i] != r->len[i])
			r->verdict[i] = V_INNER;            /* chain: the inner's checks */
	}
	if (g->rss && rss_ok)
		for (i = lo; i < hi; i++)
			if (r->verdict[i] == GCS_V_ACCEPT && r->queue[i] != (uint16_t)g->own_queue)
				g->st.rx_foreign++;
}

/* The verify of frames [lo, hi) failed: every one comes back NULL. */
static void rx_unverified(struct gthr *g, struct rx_if *r, int32_t lo, int32_t hi, int rc)
{
	int32_t i;

	gpu_failed(g, "RX verify", (uint32_t)(hi - lo), rc);
	for (i = lo; i < hi; i++) {
		if (r->ptr[i] && r->glen[i] == r->len[i])
			g->st.rx_unverified++;
		r->verdict[i] = GCS_V_DROP_TRUNC;
	}
	rx_settle(g, r, lo, hi, 0);
}

/* Verify as you go: wait until frame `index` has its verdict -- the group
 * holding it, and with it every group posted before (gcs_wait completes in
 * posting order). */
static void rx_wait(struct gthr *g, struct rx_if *r, int32_t index)
{
	const uint32_t G = g->rx_group;
	uint32_t grp = (uint32_t)index / G, k;
	int32_t hi;
	int rc = 0;

	if (grp >= r->ngroups)
		grp = r->ngroups - 1;
	for (k = grp + 1; k-- > r->ready / G;)
		if (r->ticket[k]) {                 /* the newest posted group up to grp */
			rc = gcs_wait(g->gcs, r->ticket[k]);
			break;
		}
	hi = (int32_t)((grp + 1) * G) < r->n ? (int32_t)((grp + 1) * G) : r->n;
	if (rc && r->ngroups > 0 && k + 1 < r->ngroups && r->ticket[r->ngroups - 1])
		/* the failed wait cancelled the burst's later groups too and left
		 * them to be reported by a wait that covers them: take that report
		 * here, so no wait of a later burst inherits it */
		(void)gcs_wait(g->gcs, r->ticket[r->ngroups - 1]);
	if (rc)
		rx_unverified(g, r, (int32_t)r->ready, r->n, rc);   /* the rest of the burst */
	else
		rx_settle(g, r, (int32_t)r->ready, hi, 1);
	r->ready = rc ? (uint32_t)r->n : (uint32_t)hi;
}

static int32_t gpucsum_recv_pkts(struct mtcp_thread_context *ctx, int ifidx)
{
	struct gthr *g = lookup(ctx);
	struct rx_if *r;
	int32_t n, i;
	const int chained = (g_caps & GPUCSUM_INNER_RX_CHAINED) != 0;
	int rc;

	if (g && ifidx >= 0 && ifidx < GPUCSUM_MAX_IFS && g->rx[ifidx] &&
	    g->rx[ifidx]->ready < (uint32_t)g->rx[ifidx]->n && g->rx[ifidx]->n > 0)
		/* a loop that left frames of the last burst unread: its groups
		 * complete before the inner reuses their buffers */
		rx_wait(g, g->rx[ifidx], g->rx[ifidx]->n - 1);
	n = g_inner->recv_pkts(ctx, ifidx);
	if (!g || ifidx < 0 || ifidx >= GPUCSUM_MAX_IFS)
		return n;
	if (!g->rx[ifidx])
		g->rx[ifidx] = calloc(1, sizeof(struct rx_if));
	r = g->rx[ifidx];
	if (!r)
		die("calloc", GCS_ENOMEM);
	r->n = 0;
	r->ready = 0;
	r->ngroups = 0;
	if (n <= 0)
		return n;
	if (rx_reserve(r, (uint32_t)n))
		die("RX burst arrays", GCS_ENOMEM);
	/* One pass over the inner burst to learn every frame's address.  get_rptr
	 * is called again per index when mTCP walks the burst (below), except
	 * with RX_ONCE, where this is the inner's only call. */
	for (i = 0; i < n; i++) {
		r->len[i] = 0;
		r->ptr[i] = g_inner->get_rptr(ctx, ifidx, i, &r->len[i]);
		if (!r->ptr[i])
			r->len[i] = 0;
		r->glen[i] = (chained && r->len[i] > g_seg_max) ? 0 : r->len[i];
	}
	g->st.rx_frames += (uint64_t)n;
	r->n = n;
	if (g->rx_group && !g->rss) {
		/* verify as you go: post the groups, return; get_rptr waits */
		const uint32_t G = g->rx_group;
		for (i = 0; i < n; i += (int32_t)G) {
			const uint32_t m = (uint32_t)(n - i) < G ? (uint32_t)(n - i) : G;
			uint64_t t = 0;
			rc = gcs_verify_ptrs_async(g->gcs, r->ptr + i, r->glen + i, m, r->verdict + i,
			                           GCS_VF_ZERO_BAD_TCP_CHECK, &t);
			if (rc) {
				/* the groups posted so far complete; the rest is unverified */
				if (i > 0)
					rx_wait(g, r, i - 1);
				if (r->ready < (uint32_t)n)
					rx_unverified(g, r, (int32_t)r->ready, n, rc);
				r->ready = (uint32_t)n;
				break;
			}
			r->ticket[r->ngroups++] = t;
			g->st.rx_posts++;
		}
		g->st.rx_batches++;
		return n;
	}
	if (g->rss)
		rc = gcs_classify_ptrs(g->gcs, r->ptr, r->glen, (uint32_t)n, r->verdict, NULL,
		                       r->queue, GCS_VF_ZERO_BAD_TCP_CHECK);
	else
		rc = gcs_verify_ptrs(g->gcs, r->ptr, r->glen, (uint32_t)n, r->verdict,
		                     GCS_VF_ZERO_BAD_TCP_CHECK);
	if (rc) {
		/* unverified: every frame of the burst comes back NULL */
		rx_unverified(g, r, 0, n, rc);
	} else {
		g->st.rx_batches++;
		rx_settle(g, r, 0, n, 1);
	}
	r->ready = (uint32_t)n;
	return n;
}

static uint8_t *gpucsum_get_rptr(struct mtcp_thread_context *ctx, int ifidx, int index,
                                 uint16_t *len)
{
	struct gthr *g = lookup(ctx);
	struct rx_if *r = (g && ifidx >= 0 && ifidx < GPUCSUM_MAX_IFS) ? g->rx[ifidx] : NULL;
	uint8_t *p;
	uint16_t l = 0;

	if (!r || index < 0 || index >= r->n)
		return g_inner->get_rptr(ctx, ifidx, index, len);
	if ((uint32_t)index >= r->ready)
		rx_wait(g, r, index);                   /* verify as you go */
	if (g_caps & GPUCSUM_INNER_RX_ONCE) {
		/* the burst pass's call was the inner's one call for this index */
		if (GCS_V_IS_ERROR(r->verdict[index])) {
			g->st.rx_errors++;
			return NULL;
		}
		*len = r->len[index];
		return r->ptr[index];
	}
	if (r->verdict[index] == V_INNER) {
		g->st.rx_inner++;
		p = g_inner->get_rptr(ctx, ifidx, index, len);
		if (!p)
			g->st.rx_errors++;
		return p;
	}
	if (GCS_V_IS_ERROR(r->verdict[index])) {
		g->st.rx_errors++;
		return NULL;
	}
	/* Same index again: inner per-index state now points at this frame. */
	p = g_inner->get_rptr(ctx, ifidx, index, &l);
	if (p != r->ptr[index] || l != r->len[index]) {
		g->st.rx_rptr_changed++;
		g->st.rx_errors++;
		return NULL;
	}
	*len = l;
	return p;
}

static int32_t gpucsum_select(struct mtcp_thread_context *ctx)
{
	return g_inner->select ? g_inner->select(ctx) : 0;
}

static void gpucsum_destroy_handle(struct mtcp_thread_context *ctx)
{
	struct gthr *g = lookup(ctx);
	int i;

	if (g)
		for (i = 0; i < GPUCSUM_MAX_IFS; i++)
			if (g->rx[i] && g->rx[i]->n > 0 && g->rx[i]->ready < (uint32_t)g->rx[i]->n)
				rx_wait(g, g->rx[i], g->rx[i]->n - 1);   /* nothing in flight */
	if (g_inner->destroy_handle)
		g_inner->destroy_handle(ctx);
	if (!g)
		return;
	pthread_mutex_lock(&g_lock);
	for (i = 0; i < GPUCSUM_MAX_THREADS; i++)
		if (g_table[i] == g)
			g_table[i] = NULL;
	pthread_mutex_unlock(&g_lock);
	if (t_cache == g)
		t_cache = NULL;
	if (g->gcs) {
		/* the context drains its ring and streams first: a device fault that
		 * surfaces there is this thread's, reported as a GPU failure */
		int rc = gcs_ctx_destroy(g->gcs);
		if (rc)
			gpu_failed(g, "context teardown", 0, rc);
	}
	for (i = 0; i < GPUCSUM_MAX_IFS; i++) {
		if (g->rx[i]) {
			free(g->rx[i]->ptr);
			free(g->rx[i]->len);
			free(g->rx[i]->glen);
			free(g->rx[i]->verdict);
			free(g->rx[i]->queue);
			free(g->rx[i]->ticket);
			free(g->rx[i]);
		}
		if (g->tx[i]) {
			free(g->tx[i]->shadow);
			free(g->tx[i]);
		}
	}
	free(g);
}

/* dpdk_dev_ioctl (dpdk_module.c:805-928) answers 0 when the NIC does the
 * work; here the GPU does it, in recv_pkts (RX) and send_pkts (TX). */
static int32_t gpucsum_dev_ioctl(struct mtcp_thread_context *ctx, int nif, int cmd, void *argp)
{
	switch (cmd) {
	case PKT_TX_TCPIP_CSUM:       /* tcp_out.c:206, :326               */
		/* asked after the segment's headers and payload are written: the
		 * thread's most recent get_wptr frame is complete (an ICMP frame's
		 * PKT_TX_IP_CSUM comes before its ICMP part: not a signal).  nif is
		 * the route's ifindex (sndvar->nif_out), NOT the eidx get_wptr got
		 * (CONFIG.nif_to_eidx[nif], eth_out.c:52): the two differ unless the
		 * configured ports are 0..n-1, so the queue is the one of the last
		 * get_wptr (SendTCPPacket asks right after filling the frame that
		 * IPOutput -> EthernetOutput took, tcp_out.c:244-326). */
		{
			struct gthr *g = ctx ? lookup(ctx) : NULL;
			struct tx_if *q = g ? g->last_tx : NULL;
			if (q && q->n)
				tx_complete(g, q, q->n);
		}
		return 0;
	case PKT_TX_IP_CSUM:          /* ip_out.c:91, :163 (ICMP)          */
	case PKT_RX_IP_CSUM:          /* ip_in.c:30                        */
	case PKT_RX_TCP_CSUM:         /* tcp_in.c:1227                     */
	case PKT_TX_TCPIP_CSUM_PEEK:  /* ip_out.c:88, :160                 */
		return 0;
	case PKT_TX_TCP_CSUM:         /* NIC pseudo-header mode: not ours  */
		return -1;
	default:                      /* DRV_NAME, PKT_RX_TCP_LROSEG, ...  */
		if (g_inner && g_inner->dev_ioctl)
			return g_inner->dev_ioctl(ctx, nif, cmd, argp);
		return -1;
	}
}

io_module_func gpucsum_module_func = {
	.load_module    = gpucsum_load_module,
	.init_handle    = gpucsum_init_handle,
	.link_devices   = gpucsum_link_devices,
	.release_pkt    = gpucsum_release_pkt,
	.get_wptr       = gpucsum_get_wptr,
	.send_pkts      = gpucsum_send_pkts,
	.get_rptr       = gpucsum_get_rptr,
	.recv_pkts      = gpucsum_recv_pkts,
	.select         = gpucsum_select,
	.destroy_handle = gpucsum_destroy_handle,
	.dev_ioctl      = gpucsum_dev_ioctl,
};

int gpucsum_get_stats(struct mtcp_thread_context *ctx, struct gpucsum_stats *out)
{
	struct gthr *g = lookup(ctx);

	if (!g || !out)
		return GCS_EINVAL;
	*out = g->st;
	return GCS_OK;
}

int gpucsum_rx_verdict(struct mtcp_thread_context *ctx, int ifidx, int index)
{
	struct gthr *g = lookup(ctx);
	struct rx_if *r = (g && ifidx >= 0 && ifidx < GPUCSUM_MAX_IFS) ? g->rx[ifidx] : NULL;

	if (!r || index < 0 || index >= r->n)
		return -1;
	if ((uint32_t)index >= r->ready)
		rx_wait(g, r, index);
	if (r->verdict[index] == V_INNER)
		return -1;
	return r->verdict[index];
}

int gpucsum_set_rss(struct mtcp_thread_context *ctx, const uint8_t *key, uint32_t key_len,
                    uint32_t num_queues, int endian_check, int own_queue)
{
	struct gthr *g = lookup(ctx);
	int rc;

	if (!g)
		return GCS_EINVAL;
	if (num_queues == 0) {
		g->rss = 0;
		return GCS_OK;
	}
	if (own_queue < 0 || (uint32_t)own_queue >= num_queues)
		return GCS_EINVAL;
	rc = gcs_ctx_set_rss(g->gcs, key, key_len, num_queues, endian_check);
	if (rc)
		return rc;
	g->rss = 1;
	g->own_queue = own_queue;
	return GCS_OK;
}

int gpucsum_rx_queue(struct mtcp_thread_context *ctx, int ifidx, int index)
{
	struct gthr *g = lookup(ctx);
	struct rx_if *r = (g && ifidx >= 0 && ifidx < GPUCSUM_MAX_IFS) ? g->rx[ifidx] : NULL;

	if (!r || !g->rss || index < 0 || index >= r->n)
		return -1;
	return r->verdict[index] == GCS_V_ACCEPT ? r->queue[index] : 0xFFFF;
}
