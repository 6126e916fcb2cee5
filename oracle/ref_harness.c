#define _GNU_SOURCE
/*
 * ref_harness.c -- drives the REFERENCE's own checksum code (test
 * infrastructure only; see csum_ref.h for the rules on oracle/).
 *
 * Built by oracle/Makefile into oracle/_ref/libref_mtcp_csum.so, linking
 *   - TCPCalcChecksum from /root/reference/mtcp/src/tcp_util.c (compiled in
 *     place with the reference's flags, mtcp/src/Makefile.in:44,50,63-65), and
 *   - ip_fast_csum, the static inline x86 asm from
 *     /root/reference/io_engine/include/ps.h:66-95 (included, not copied).
 * Also ICMPChecksum (mtcp/src/icmp.c:18-42) and GetRSSHash (mtcp/src/rss.c:44-86),
 * both `static` there: oracle/Makefile compiles icmp.c / rss.c in place with
 * -fkeep-static-functions and makes just those two symbols global with
 * objcopy (no source is changed or copied), plus GetRSSCPUCore (rss.c:97-115).
 * The RX/TX drivers below follow ip_in.c:21-59 / tcp_in.c:1208-1241 and
 * ip_out.c:143-173 / tcp_out.c:244,323-333, using the same <netinet/*.h>
 * structs the reference uses, so field parsing is checked independently of
 * oracle/csum_ref.c.  Used to (1) generate tests/golden/ vectors and (2) time
 * the reference itself as bench.py's cpu_baseline ("kind": "reference").
 */
#include <stdint.h>
#include <string.h>
#include <pthread.h>
#include <arpa/inet.h>
#include <netinet/ip.h>
#include <netinet/tcp.h>
#include <netinet/ip_icmp.h>
#include <linux/if_ether.h>

#include "ps.h"   /* reference: io_engine/include/ps.h (ip_fast_csum) */

/* reference: mtcp/src/include/tcp_util.h:41-42 */
uint16_t TCPCalcChecksum(uint16_t *buf, uint16_t len, uint32_t saddr, uint32_t daddr);

uint16_t refx_tcp_calc_checksum(const uint8_t *buf, uint16_t len, uint32_t saddr,
                                uint32_t daddr)
{
	return TCPCalcChecksum((uint16_t *)buf, len, saddr, daddr);
}

uint16_t refx_ip_fast_csum(const uint8_t *iph, unsigned int ihl)
{
	return (uint16_t)ip_fast_csum(iph, ihl);
}

/* reference: mtcp/src/icmp.c:18-19, rss.c:44-45 (static, globalized), rss.h:7-9 */
uint16_t ICMPChecksum(uint16_t *icmph, int len);
uint32_t GetRSSHash(in_addr_t sip, in_addr_t dip, in_port_t sp, in_port_t dp);
int GetRSSCPUCore(in_addr_t sip, in_addr_t dip, in_port_t sp, in_port_t dp, int num_queues,
                  uint8_t endian_check);

uint16_t refx_icmp_checksum(const uint8_t *buf, int len)
{
	return ICMPChecksum((uint16_t *)buf, len);
}

uint32_t refx_rss_hash(uint32_t sip, uint32_t dip, uint16_t sp, uint16_t dp)
{
	return GetRSSHash(sip, dip, sp, dp);
}

int refx_rss_core(uint32_t sip, uint32_t dip, uint16_t sp, uint16_t dp, int num_queues,
                  int endian_check)
{
	return GetRSSCPUCore(sip, dip, sp, dp, num_queues, (uint8_t)endian_check);
}

/* Verdict codes: identical numbering to oracle/csum_ref.h REF_V_*.
 * flags & 0x2 (REF_VF_ICMP): ICMP frames are classified by ICMPChecksum. */
int refx_rx_verdict_f(uint8_t *pkt, uint32_t len, uint32_t flags)
{
	struct ethhdr *ethh = (struct ethhdr *)pkt;
	struct iphdr *iph;
	struct tcphdr *tcph;
	int ip_len, payloadlen;

	if (len < 14)
		return 8;
	if (ntohs(ethh->h_proto) != ETH_P_IP)                 /* eth_in.c:35 */
		return 1;
	if (len < 34)
		return 8;
	iph = (struct iphdr *)(pkt + sizeof(struct ethhdr));  /* ip_in.c:20 */
	ip_len = ntohs(iph->tot_len);                          /* ip_in.c:21 */
	if (ip_len < (int)sizeof(struct iphdr))                /* ip_in.c:25 */
		return 2;
	if (iph->ihl >= 5 && 14u + 4u * iph->ihl > len)
		return 8;
	if (ip_fast_csum(iph, iph->ihl))                       /* ip_in.c:35 */
		return 3;
	if (iph->version != 0x4)                               /* ip_in.c:47 */
		return 4;
	if (iph->protocol == IPPROTO_ICMP && (flags & 0x2u)) { /* ip_in.c:56 */
		int icmp_len = ip_len - (iph->ihl << 2);         /* icmp.c:89 */
		if (icmp_len >= 0 && 14u + (uint32_t)ip_len > len)
			return 8;
		return ICMPChecksum((uint16_t *)((uint8_t *)iph + (iph->ihl << 2)), icmp_len)
		           ? 11 : 10;
	}
	if (iph->protocol != IPPROTO_TCP)                      /* ip_in.c:52-59 */
		return 5;
	if (14u + (iph->ihl << 2) + 13u > len)
		return 8;
	tcph = (struct tcphdr *)((uint8_t *)iph + (iph->ihl << 2));   /* tcp_in.c:1208 */
	payloadlen = ip_len - ((iph->ihl << 2) + (tcph->doff << 2));  /* tcp_in.c:1210 */
	if (ip_len < ((iph->ihl + tcph->doff) << 2))           /* tcp_in.c:1221 */
		return 6;
	if (14u + (uint32_t)ip_len > len)
		return 8;
	if (TCPCalcChecksum((uint16_t *)tcph, (tcph->doff << 2) + payloadlen,
	                    iph->saddr, iph->daddr))           /* tcp_in.c:1231-1234 */
		return 7;
	return 0;
}

int refx_rx_verdict(uint8_t *pkt, uint32_t len)
{
	return refx_rx_verdict_f(pkt, len, 0);
}

/* TX fill (status numbering = REF_TX_*).  flags & 0x2 (REF_CF_ICMP): ICMP
 * frames also get the ICMP check, in ICMPOutput's order (icmp.c:57-69). */
int refx_tx_fill_f(uint8_t *pkt, uint32_t len, uint32_t *csums, uint32_t flags)
{
	struct ethhdr *ethh = (struct ethhdr *)pkt;
	struct iphdr *iph;
	struct tcphdr *tcph;
	int ip_len;

	if (csums)
		*csums = 0;
	if (len < 14 || ntohs(ethh->h_proto) != ETH_P_IP)
		return 2;
	if (len < 34)
		return 3;
	iph = (struct iphdr *)(pkt + sizeof(struct ethhdr));
	if (iph->ihl < 5 || 14u + 4u * iph->ihl > len)
		return 3;
	ip_len = ntohs(iph->tot_len);
	iph->check = 0;                                        /* ip_out.c:153 */
	iph->check = ip_fast_csum(iph, iph->ihl);              /* ip_out.c:172 */
	if (csums)
		*csums = iph->check;
	if (iph->protocol == IPPROTO_ICMP && (flags & 0x2u)) {
		struct icmphdr *icmph = (struct icmphdr *)((uint8_t *)iph + (iph->ihl << 2));
		if (ip_len < (int)(iph->ihl << 2) + 8 || 14u + (uint32_t)ip_len > len)
			return 6;
		icmph->checksum = 0;                               /* icmp.c:60 */
		icmph->checksum = ICMPChecksum((uint16_t *)icmph,
		                               ip_len - (iph->ihl << 2)); /* icmp.c:68-69 */
		if (csums)
			*csums = (uint32_t)iph->check | ((uint32_t)icmph->checksum << 16);
		return 5;
	}
	if (iph->protocol != IPPROTO_TCP)
		return 1;
	if (ip_len < (int)(iph->ihl << 2) + 20 || 14u + (uint32_t)ip_len > len)
		return 4;
	tcph = (struct tcphdr *)((uint8_t *)iph + (iph->ihl << 2));
	tcph->check = 0;                                       /* tcp_out.c:244 */
	tcph->check = TCPCalcChecksum((uint16_t *)tcph, ip_len - (iph->ihl << 2),
	                              iph->saddr, iph->daddr); /* tcp_out.c:330 */
	if (csums)
		*csums = (uint32_t)iph->check | ((uint32_t)tcph->check << 16);
	return 0;
}

int refx_tx_fill(uint8_t *pkt, uint32_t len, uint32_t *csums)
{
	return refx_tx_fill_f(pkt, len, csums, 0);
}

void refx_verify_fixed(uint8_t *buf, uint64_t stride, uint32_t frame_len,
                       uint32_t n, uint8_t *verdict)
{
	uint32_t i;
	for (i = 0; i < n; i++)
		verdict[i] = (uint8_t)refx_rx_verdict(buf + (uint64_t)i * stride, frame_len);
}

void refx_compute_fixed(uint8_t *buf, uint64_t stride, uint32_t frame_len,
                        uint32_t n, uint8_t *status)
{
	uint32_t i;
	for (i = 0; i < n; i++) {
		int s = refx_tx_fill(buf + (uint64_t)i * stride, frame_len, NULL);
		if (status)
			status[i] = (uint8_t)s;
	}
}

struct rshard {
	uint8_t *buf;
	uint64_t stride;
	uint32_t frame_len, lo, hi;
	uint8_t *out;
	int compute;
};

static void *rshard_main(void *arg)
{
	struct rshard *s = (struct rshard *)arg;
	uint8_t *base = s->buf + (uint64_t)s->lo * s->stride;
	if (s->compute)
		refx_compute_fixed(base, s->stride, s->frame_len, s->hi - s->lo,
		                   s->out ? s->out + s->lo : NULL);
	else
		refx_verify_fixed(base, s->stride, s->frame_len, s->hi - s->lo,
		                  s->out + s->lo);
	return NULL;
}

/* Independent frame shards, one pthread per shard (mTCP's per-core model). */
void refx_run_fixed_mt(uint8_t *buf, uint64_t stride, uint32_t frame_len,
                       uint32_t n, uint8_t *out, int compute, int threads)
{
	enum { MAXT = 256 };
	pthread_t tid[MAXT];
	int live[MAXT];
	struct rshard sh[MAXT];
	int t;

	if (threads < 1)
		threads = 1;
	if (threads > MAXT)
		threads = MAXT;
	for (t = 0; t < threads; t++) {
		sh[t].buf = buf;
		sh[t].stride = stride;
		sh[t].frame_len = frame_len;
		sh[t].lo = (uint32_t)((uint64_t)n * t / threads);
		sh[t].hi = (uint32_t)((uint64_t)n * (t + 1) / threads);
		sh[t].out = out;
		sh[t].compute = compute;
	}
	for (t = 1; t < threads; t++) {
		live[t] = pthread_create(&tid[t], NULL, rshard_main, &sh[t]) == 0;
		if (!live[t])
			rshard_main(&sh[t]);
	}
	rshard_main(&sh[0]);
	for (t = 1; t < threads; t++)
		if (live[t])
			pthread_join(tid[t], NULL);
}

/* The same shards, each on a thread pinned to cpus[t] before it starts
 * (1 pinned core, and one thread per host core).  The caller's
 * own affinity is left alone: it only waits. */
int refx_run_fixed_pinned(uint8_t *buf, uint64_t stride, uint32_t frame_len, uint32_t n,
                          uint8_t *out, int compute, int threads, const int *cpus)
{
	enum { MAXT = 256 };
	pthread_t tid[MAXT];
	struct rshard sh[MAXT];
	int t, rc = 0;

	if (threads < 1 || threads > MAXT || !cpus)
		return -1;
	for (t = 0; t < threads; t++) {
		pthread_attr_t at;
		cpu_set_t set;
		sh[t].buf = buf;
		sh[t].stride = stride;
		sh[t].frame_len = frame_len;
		sh[t].lo = (uint32_t)((uint64_t)n * t / threads);
		sh[t].hi = (uint32_t)((uint64_t)n * (t + 1) / threads);
		sh[t].out = out;
		sh[t].compute = compute;
		CPU_ZERO(&set);
		CPU_SET(cpus[t], &set);
		pthread_attr_init(&at);
		pthread_attr_setaffinity_np(&at, sizeof(set), &set);
		if (pthread_create(&tid[t], &at, rshard_main, &sh[t]) != 0) {
			pthread_attr_destroy(&at);
			threads = t;
			rc = -1;
			break;
		}
		pthread_attr_destroy(&at);
	}
	for (t = 0; t < threads; t++)
		pthread_join(tid[t], NULL);
	return rc;
}
