/*
 * csum_ref.c -- CPU ORACLE (test infrastructure only; see csum_ref.h).
 *
 * Clean-room restatement of mTCP's --disable-hwcsum checksum path.  Compiled
 * with the reference's own flags (-O3 -g -DNDEBUG -m64 -fgnu89-inline,
 * mtcp/src/Makefile.in:44,50) so that it doubles as the "port" CPU baseline.
 */
#include "csum_ref.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* Little-endian loads from any alignment (the reference dereferences
 * uint16_t* / u32* on x86, which is little-endian and unaligned-tolerant). */
static inline uint32_t ld16(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
static inline uint32_t ld32(const uint8_t *p)
{
	return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
	       ((uint32_t)p[3] << 24);
}
static inline uint16_t bswap16(uint16_t v) { return (uint16_t)((v >> 8) | (v << 8)); }

/* tcp_util.c:244-277.  32-bit accumulator of little-endian 16-bit words,
 * odd tail = low byte of the last word (mask ntohs(0xFF00) == 0x00FF on LE,
 * :262-263), pseudo-header halves of saddr/daddr as stored, htons(len),
 * htons(IPPROTO_TCP), two-step fold (:271-272), complement (:274). */
uint16_t ref_tcp_calc_checksum(const uint8_t *buf, uint16_t len,
                               uint32_t saddr, uint32_t daddr)
{
	uint32_t sum = 0;
	int nleft = len;
	const uint8_t *w = buf;

	while (nleft > 1) {
		sum += ld16(w);
		w += 2;
		nleft -= 2;
	}
	if (nleft)
		sum += w[0];            /* == *w & 0x00FF */

	sum += (saddr & 0x0000FFFFu) + (saddr >> 16);
	sum += (daddr & 0x0000FFFFu) + (daddr >> 16);
	sum += bswap16(len);
	sum += bswap16(6);          /* IPPROTO_TCP */

	sum = (sum >> 16) + (sum & 0xFFFFu);
	sum += (sum >> 16);
	return (uint16_t)~sum;
}

/* ps.h:66-95, the x86 asm actually used on x86_64 builds:
 *   movl (iph),sum ; subl $4,ihl ; jbe 2f   -> ihl<=4: raw low 16 bits of word 0
 *   addl 4 ; adcl 8 ; adcl 12 ; loop adcl 16.. (ihl-4 times) ; adcl $0
 *   fold: (sum>>16) +w low16(sum) with carry ; notl */
uint16_t ref_ip_fast_csum(const uint8_t *iph, unsigned int ihl)
{
	uint32_t sum = ld32(iph);
	uint64_t t;
	uint32_t c;
	unsigned int k;

	if (ihl <= 4)
		return (uint16_t)sum;

	t = (uint64_t)sum + ld32(iph + 4);
	sum = (uint32_t)t;
	c = (uint32_t)(t >> 32);
	for (k = 2; k < ihl; k++) {
		t = (uint64_t)sum + ld32(iph + 4 * k) + c;
		sum = (uint32_t)t;
		c = (uint32_t)(t >> 32);
	}
	sum += c;                    /* adcl $0 (a carry out here is dropped) */

	{
		uint32_t r = (sum >> 16) + (sum & 0xFFFFu);   /* addw */
		sum = (r & 0xFFFFu) + (r >> 16);               /* adcl $0 */
	}
	return (uint16_t)~sum;
}

/* icmp.c:18-42.  Same word loop as TCPCalcChecksum without a pseudo header;
 * the odd final byte is the low byte of a word whose high byte the C leaves
 * uninitialised -- zero here, as in the reference's gcc -O3 object (movzbl),
 * pinned by tests/golden/icmp_fn.npz. */
uint16_t ref_icmp_checksum(const uint8_t *buf, int len)
{
	uint32_t sum = 0;
	const uint8_t *w = buf;

	while (len > 1) {
		sum += ld16(w);
		w += 2;
		len -= 2;
	}
	if (len == 1)
		sum += w[0];
	sum = (sum >> 16) + (sum & 0xFFFFu);
	sum += (sum >> 16);
	return (uint16_t)~sum;
}

/* rss.c:19-25: the key mTCP's RSS address selection assumes. */
const uint8_t REF_RSS_DEFAULT_KEY[40] = {
	5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5,
	5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5};

/* rss.c:13-41: cache[i] = the 32 key bits starting at bit i (MSB-first). */
void ref_rss_key_cache(const uint8_t *key, uint32_t cache[96])
{
	int i;
	if (!key)
		key = REF_RSS_DEFAULT_KEY;
	for (i = 0; i < 96; i++) {
		uint32_t v = 0;
		int b;
		for (b = 0; b < 32; b++) {
			int bit = i + b;
			v = (v << 1) | ((key[bit >> 3] >> (7 - (bit & 7))) & 1u);
		}
		cache[i] = v;
	}
}

/* rss.c:44-86: Toeplitz hash, input bits MSB-first: sip, dip, sp, dp. */
uint32_t ref_rss_hash(const uint8_t *key, uint32_t sip, uint32_t dip, uint16_t sp,
                      uint16_t dp)
{
	uint32_t cache[96], h = 0;
	int i;
	ref_rss_key_cache(key, cache);
	for (i = 0; i < 32; i++)
		if ((sip >> (31 - i)) & 1u)
			h ^= cache[i];
	for (i = 0; i < 32; i++)
		if ((dip >> (31 - i)) & 1u)
			h ^= cache[32 + i];
	for (i = 0; i < 16; i++)
		if ((sp >> (15 - i)) & 1u)
			h ^= cache[64 + i];
	for (i = 0; i < 16; i++)
		if ((dp >> (15 - i)) & 1u)
			h ^= cache[80 + i];
	return h;
}

/* rss.c:97-115 */
int ref_rss_core(const uint8_t *key, uint32_t sip, uint32_t dip, uint16_t sp, uint16_t dp,
                 int num_queues, int endian_check)
{
	static const uint32_t adj[4] = {3u, 1u, 0xFFFFFFFFu, 0xFFFFFFFDu};
	uint32_t m;
	if (endian_check) {
		m = ref_rss_hash(key, sip, dip, sp, dp) & 0x1FFu;
		m += adj[m & 3u];
	} else {
		m = ref_rss_hash(key, sip, dip, sp, dp) & 0x7Fu;
	}
	return (int)(m % (uint32_t)num_queues);
}

/* RX verdict in the reference's order:
 *   eth_in.c:35  ethertype == ETH_P_IP, else ARP/release (not checked)
 *   ip_in.c:21-26  ip_len = ntohs(tot_len); ip_len < 20 -> ERROR
 *   ip_in.c:35-36  ip_fast_csum(iph, ihl) != 0 -> ERROR
 *   ip_in.c:47-50  version != 4 -> release, FALSE
 *   ip_in.c:52-59  protocol: TCP -> ProcessTCPPacket, else not TCP
 *   tcp_in.c:1221-1222  ip_len < (ihl+doff)<<2 -> ERROR
 *   tcp_in.c:1231-1239  TCPCalcChecksum(tcph, doff*4+payloadlen = ip_len-ihl*4,
 *                       saddr, daddr) != 0 -> tcph->check = 0, ERROR
 * Reads the reference would make past `len` (undefined there) are DROP_TRUNC
 * here; everything the reference can compute in-bounds is reproduced as is. */
int ref_rx_verdict(uint8_t *f, uint32_t len, uint32_t flags)
{
	uint32_t ihl, version, proto, tot_len, doff, ts, tcplen;
	uint8_t *iph, *tcph;

	if (len < 14)
		return REF_V_DROP_TRUNC;
	if (ld16(f + 12) != 0x0008)              /* ntohs(h_proto) != 0x0800 */
		return REF_V_NOT_IPV4;
	if (len < 34)
		return REF_V_DROP_TRUNC;
	iph = f + 14;
	ihl = iph[0] & 0x0F;
	version = iph[0] >> 4;
	tot_len = bswap16((uint16_t)ld16(iph + 2));
	proto = iph[9];
	if (tot_len < 20)
		return REF_V_DROP_IPLEN;
	if (ihl >= 5 && 14 + 4 * ihl > len)
		return REF_V_DROP_TRUNC;
	if (ref_ip_fast_csum(iph, ihl) != 0)
		return REF_V_DROP_IPCSUM;
	if (version != 4)
		return REF_V_NOT_V4;
	if (proto == 1 && (flags & REF_VF_ICMP)) {
		/* ProcessICMPPacket (ip_in.c:56) -> ICMPChecksum(icmph, ip_len - ihl*4)
		 * (icmp.c:89); a negative length sums nothing (0xFFFF: bad). */
		if (tot_len < 4 * ihl)
			return REF_V_ICMP_BADCSUM;
		if (14 + tot_len > len)
			return REF_V_DROP_TRUNC;
		return ref_icmp_checksum(iph + 4 * ihl, (int)(tot_len - 4 * ihl)) != 0
		           ? REF_V_ICMP_BADCSUM
		           : REF_V_ICMP_OK;
	}
	if (proto != 6)
		return REF_V_NOT_TCP;
	ts = 14 + 4 * ihl;
	if (ts + 13 > len)                       /* doff byte lies past the frame */
		return REF_V_DROP_TRUNC;
	tcph = f + ts;
	doff = tcph[12] >> 4;
	if (tot_len < 4 * (ihl + doff))
		return REF_V_DROP_TCPLEN;
	if (14 + tot_len > len)
		return REF_V_DROP_TRUNC;
	tcplen = tot_len - 4 * ihl;
	if (ref_tcp_calc_checksum(tcph, (uint16_t)tcplen, ld32(iph + 12),
	                          ld32(iph + 16)) != 0) {
		if ((flags & REF_VF_ZERO_BAD_TCP_CHECK) && ts + 18 <= len) {
			tcph[16] = 0;
			tcph[17] = 0;
		}
		return REF_V_DROP_TCPCSUM;
	}
	return REF_V_ACCEPT;
}

/* TX fill, mTCP order: IPOutput sets iph->check = 0 then stores
 * ip_fast_csum(iph, ihl) (ip_out.c:153, :172); SendTCPPacket memsets the TCP
 * header (check = 0, tcp_out.c:244) and stores TCPCalcChecksum(tcph,
 * 20+optlen+payloadlen = tot_len - ihl*4, saddr, daddr) (tcp_out.c:323-333).
 * Non-TCP IPv4 frames get only the IP check (ICMP: ip_out.c:90-92,100). */
int ref_tx_fill(uint8_t *f, uint32_t len, uint32_t *csums)
{
	return ref_tx_fill_f(f, len, csums, 0);
}

int ref_tx_fill_f(uint8_t *f, uint32_t len, uint32_t *csums, uint32_t flags)
{
	uint32_t ihl, proto, tot_len, ts;
	uint16_t ipc, tcpc;
	uint8_t *iph, *tcph;

	if (csums)
		*csums = 0;
	if (len < 14 || ld16(f + 12) != 0x0008)
		return REF_TX_NOT_IPV4;
	if (len < 34)
		return REF_TX_BAD_HDR;
	iph = f + 14;
	ihl = iph[0] & 0x0F;
	if (ihl < 5 || 14 + 4 * ihl > len)
		return REF_TX_BAD_HDR;
	tot_len = bswap16((uint16_t)ld16(iph + 2));
	proto = iph[9];

	iph[10] = 0;
	iph[11] = 0;
	ipc = ref_ip_fast_csum(iph, ihl);
	memcpy(iph + 10, &ipc, 2);
	if (csums)
		*csums = ipc;
	if (proto == 1 && (flags & REF_CF_ICMP)) {
		/* ICMPOutput (icmp.c:44-77): icmp_checksum = 0, then ICMPChecksum over
		 * sizeof(struct icmphdr) + len = tot_len - ihl*4 bytes. */
		uint8_t *icmph = iph + 4 * ihl;
		uint16_t icc;
		if (tot_len < 4 * ihl + 8 || 14 + tot_len > len)
			return REF_TX_BAD_ICMPLEN;
		icmph[2] = 0;
		icmph[3] = 0;
		icc = ref_icmp_checksum(icmph, (int)(tot_len - 4 * ihl));
		memcpy(icmph + 2, &icc, 2);
		if (csums)
			*csums = (uint32_t)ipc | ((uint32_t)icc << 16);
		return REF_TX_ICMP_OK;
	}
	if (proto != 6)
		return REF_TX_IP_ONLY;
	ts = 4 * ihl;
	if (tot_len < ts + 20 || 14 + tot_len > len)
		return REF_TX_BAD_TCPLEN;
	tcph = iph + ts;
	tcph[16] = 0;
	tcph[17] = 0;
	tcpc = ref_tcp_calc_checksum(tcph, (uint16_t)(tot_len - ts), ld32(iph + 12),
	                             ld32(iph + 16));
	memcpy(tcph + 16, &tcpc, 2);
	if (csums)
		*csums = (uint32_t)ipc | ((uint32_t)tcpc << 16);
	return REF_TX_OK;
}

/* tcp_out.c:316-321 memcpy's the payload behind header + options, then
 * :323-333 folds; IPOutput's fold follows (ip_out.c:172). */
int ref_tx_copy_fill(uint8_t *f, uint32_t len, const uint8_t *src, uint64_t src_avail,
                     uint32_t *csums)
{
	if (len >= 34 && ld16(f + 12) == 0x0008) {
		uint32_t ihl = f[14] & 0x0Fu, ts = 14 + 4 * ihl;
		uint32_t tot = bswap16((uint16_t)ld16(f + 16));
		if (ihl >= 5 && f[23] == 6 && ts + 12 < len) {
			uint32_t doff = f[ts + 12] >> 4, hl = ts + 4 * doff;
			if (doff >= 5 && tot >= 4 * (ihl + doff) && 14 + tot <= len) {
				uint32_t plen = 14 + tot - hl;
				if (!src || plen > src_avail) {
					if (csums)
						*csums = 0;
					return REF_TX_BAD_DESC;
				}
				memcpy(f + hl, src, plen);
			}
		}
	}
	return ref_tx_fill(f, len, csums);
}

void ref_compute_copy_batch(uint8_t *buf, uint64_t buf_bytes, const uint64_t *off,
                            const uint16_t *len, uint32_t n, const uint8_t *src,
                            uint64_t src_bytes, const uint64_t *src_off, uint8_t *status,
                            uint32_t *csums)
{
	uint32_t i;
	for (i = 0; i < n; i++) {
		int s;
		uint64_t so = src_off[i];
		if (!((off[i] & 15) == 0 && off[i] <= buf_bytes && len[i] <= buf_bytes - off[i])) {
			s = REF_TX_BAD_DESC;
			if (csums)
				csums[i] = 0;
		} else {
			s = ref_tx_copy_fill(buf + off[i], len[i], so <= src_bytes ? src + so : NULL,
			                     so <= src_bytes ? src_bytes - so : 0,
			                     csums ? &csums[i] : NULL);
		}
		if (status)
			status[i] = (uint8_t)s;
	}
}

/* ---- software LRO (see csum_ref.h) --------------------------------------- */

static uint32_t be16(const uint8_t *p) { return ((uint32_t)p[0] << 8) | p[1]; }
static uint32_t be32(const uint8_t *p)
{
	return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* TCP payload bytes of an ACCEPT frame with ihl == 5, else -1 */
static int gro_payload(const uint8_t *f)
{
	uint32_t doff = f[46] >> 4, tot = be16(f + 16);
	if ((f[14] & 0x0F) != 5)
		return -1;
	return (int)tot - 20 - 4 * (int)doff;
}

static int gro_continues(const uint8_t *p, const uint8_t *c)
{
	int pp = gro_payload(p), pc = gro_payload(c);
	uint32_t doff = p[46] >> 4, k;
	if (pp <= 0 || pc <= 0)
		return 0;
	if (p[15] != c[15] || be16(p + 20) != be16(c + 20) || (be16(p + 20) & 0x3FFF) ||
	    p[22] != c[22] || memcmp(p + 26, c + 26, 8))
		return 0;
	if (be16(c + 18) != be16(p + 18) && be16(c + 18) != ((be16(p + 18) + 1) & 0xFFFF))
		return 0;
	if (memcmp(p + 34, c + 34, 4) || memcmp(p + 42, c + 42, 4) || c[46] != p[46] ||
	    (p[46] & 0x0F) || be16(p + 48) != be16(c + 48) || be16(p + 52) || be16(c + 52))
		return 0;
	if (p[47] != 0x10 || (c[47] != 0x10 && c[47] != 0x18))
		return 0;
	for (k = 54; k < 34 + 4 * doff; k++)
		if (p[k] != c[k])
			return 0;
	return be32(c + 38) == be32(p + 38) + (uint32_t)pp;
}

void ref_gro_batch(const uint8_t *buf, uint64_t buf_bytes, const uint64_t *off,
                   const uint16_t *len, const uint8_t *verdict, uint32_t n,
                   uint32_t window, uint32_t max_len, uint8_t *out, uint64_t out_bytes,
                   uint64_t *out_off, uint16_t *out_len, uint32_t *head)
{
	uint32_t w0, i;
	if (window == 0)
		window = 1;
	for (w0 = 0; w0 < n; w0 += window) {
		uint32_t w1 = w0 + window < n ? w0 + window : n;
		uint64_t o = off[w0];
		i = w0;
		while (i < w1) {
			/* run [i, j) */
			const uint8_t *h = buf + off[i];
			uint32_t j = i + 1, mlen;
			if (verdict[i] == REF_V_ACCEPT && (off[i] & 15) == 0 && off[i] <= buf_bytes &&
			    len[i] <= buf_bytes - off[i] && gro_payload(h) > 0) {
				uint32_t hl = 34 + 4 * (h[46] >> 4);
				mlen = hl + (uint32_t)gro_payload(h);
				while (j < w1 && verdict[j] == REF_V_ACCEPT && (off[j] & 15) == 0 &&
				       off[j] <= buf_bytes && len[j] <= buf_bytes - off[j] &&
				       gro_continues(buf + off[j - 1], buf + off[j]) &&
				       mlen + (uint32_t)gro_payload(buf + off[j]) <= max_len) {
					mlen += (uint32_t)gro_payload(buf + off[j]);
					j++;
				}
			}
			head[i] = i;
			out_off[i] = o;
			if (j == i + 1) {
				/* a single frame: copied as it is (a bad descriptor: nothing) */
				int ok = (off[i] & 15) == 0 && off[i] <= buf_bytes &&
				         len[i] <= buf_bytes - off[i];
				out_len[i] = ok ? len[i] : 0;
				if (ok && o < out_bytes)
					memcpy(out + o, h, o + len[i] <= out_bytes ? len[i] : out_bytes - o);
			} else {
				uint32_t hl = 34 + 4 * (h[46] >> 4), k, pos = hl, psh = 0;
				uint8_t *m = (uint8_t *)malloc(mlen);
				out_len[i] = (uint16_t)mlen;
				memcpy(m, h, hl);
				for (k = i; k < j; k++) {
					const uint8_t *f = buf + off[k];
					uint32_t pl = (uint32_t)gro_payload(f);
					memcpy(m + pos, f + hl, pl);
					pos += pl;
					psh |= f[47] & 0x08;
					if (k > i) {
						head[k] = i;
						out_off[k] = o;
						out_len[k] = 0;
					}
				}
				m[16] = (uint8_t)((mlen - 14) >> 8);
				m[17] = (uint8_t)(mlen - 14);
				m[47] |= (uint8_t)psh;
				ref_tx_fill(m, mlen, NULL);
				if (o < out_bytes)
					memcpy(out + o, m, o + mlen <= out_bytes ? mlen : out_bytes - o);
				free(m);
			}
			o += (out_len[i] + 15u) & ~15ull;
			i = j;
		}
	}
}

static int desc_ok(uint64_t buf_bytes, uint64_t off, uint32_t len)
{
	return (off & 15) == 0 && off <= buf_bytes && len <= buf_bytes - off;
}

void ref_verify_batch(uint8_t *buf, uint64_t buf_bytes, const uint64_t *off,
                      const uint16_t *len, uint32_t n, uint8_t *verdict,
                      uint32_t flags)
{
	uint32_t i;
	for (i = 0; i < n; i++)
		verdict[i] = desc_ok(buf_bytes, off[i], len[i])
		                 ? (uint8_t)ref_rx_verdict(buf + off[i], len[i], flags)
		                 : REF_V_BAD_DESC;
}

void ref_compute_batch(uint8_t *buf, uint64_t buf_bytes, const uint64_t *off,
                       const uint16_t *len, uint32_t n, uint8_t *status,
                       uint32_t *csums)
{
	ref_compute_batch_f(buf, buf_bytes, off, len, n, status, csums, 0);
}

/* Steering of one verdict (ref_classify_*): ACCEPT frames only. */
static void classify_one(const uint8_t *f, int vd, uint32_t *hash, uint16_t *queue,
                         const uint8_t *key, int num_queues, int endian_check)
{
	uint32_t ts, sip, dip;
	uint16_t sp, dp;
	if (vd != REF_V_ACCEPT) {
		if (hash)
			*hash = 0;
		if (queue)
			*queue = 0xFFFF;
		return;
	}
	ts = 14 + 4 * (f[14] & 0x0Fu);
	sip = ((uint32_t)f[26] << 24) | ((uint32_t)f[27] << 16) | ((uint32_t)f[28] << 8) | f[29];
	dip = ((uint32_t)f[30] << 24) | ((uint32_t)f[31] << 16) | ((uint32_t)f[32] << 8) | f[33];
	sp = (uint16_t)((f[ts] << 8) | f[ts + 1]);
	dp = (uint16_t)((f[ts + 2] << 8) | f[ts + 3]);
	if (hash)
		*hash = ref_rss_hash(key, sip, dip, sp, dp);
	if (queue)
		*queue = (uint16_t)ref_rss_core(key, sip, dip, sp, dp, num_queues, endian_check);
}

void ref_classify_batch(uint8_t *buf, uint64_t buf_bytes, const uint64_t *off,
                        const uint16_t *len, uint32_t n, uint8_t *verdict,
                        uint32_t *hash, uint16_t *queue, uint32_t flags,
                        const uint8_t *key, int num_queues, int endian_check)
{
	uint32_t i;
	ref_verify_batch(buf, buf_bytes, off, len, n, verdict, flags);
	for (i = 0; i < n; i++)
		classify_one(verdict[i] == REF_V_BAD_DESC ? NULL : buf + off[i], verdict[i],
		             hash ? hash + i : NULL, queue ? queue + i : NULL, key, num_queues,
		             endian_check);
}

void ref_classify_fixed(uint8_t *buf, uint64_t stride, uint32_t frame_len, uint32_t n,
                        uint8_t *verdict, uint32_t *hash, uint16_t *queue,
                        uint32_t flags, const uint8_t *key, int num_queues,
                        int endian_check)
{
	uint32_t i;
	ref_verify_fixed(buf, stride, frame_len, n, verdict, flags);
	for (i = 0; i < n; i++)
		classify_one(buf + (uint64_t)i * stride, verdict[i], hash ? hash + i : NULL,
		             queue ? queue + i : NULL, key, num_queues, endian_check);
}

void ref_compute_batch_f(uint8_t *buf, uint64_t buf_bytes, const uint64_t *off,
                         const uint16_t *len, uint32_t n, uint8_t *status,
                         uint32_t *csums, uint32_t flags)
{
	uint32_t i;
	for (i = 0; i < n; i++) {
		int s;
		if (!desc_ok(buf_bytes, off[i], len[i])) {
			s = REF_TX_BAD_DESC;
			if (csums)
				csums[i] = 0;
		} else {
			s = ref_tx_fill_f(buf + off[i], len[i], csums ? &csums[i] : NULL, flags);
		}
		if (status)
			status[i] = (uint8_t)s;
	}
}

void ref_verify_fixed(uint8_t *buf, uint64_t stride, uint32_t frame_len,
                      uint32_t n, uint8_t *verdict, uint32_t flags)
{
	uint32_t i;
	for (i = 0; i < n; i++)
		verdict[i] = (uint8_t)ref_rx_verdict(buf + (uint64_t)i * stride, frame_len, flags);
}

void ref_compute_fixed(uint8_t *buf, uint64_t stride, uint32_t frame_len,
                       uint32_t n, uint8_t *status, uint32_t *csums)
{
	uint32_t i;
	for (i = 0; i < n; i++) {
		int s = ref_tx_fill(buf + (uint64_t)i * stride, frame_len,
		                    csums ? &csums[i] : NULL);
		if (status)
			status[i] = (uint8_t)s;
	}
}

struct shard {
	uint8_t *buf;
	uint64_t stride;
	uint32_t frame_len, lo, hi, flags;
	uint8_t *out;
	uint32_t *csums;
	int compute;
};

static void *shard_main(void *arg)
{
	struct shard *s = (struct shard *)arg;
	uint8_t *base = s->buf + (uint64_t)s->lo * s->stride;
	uint32_t cnt = s->hi - s->lo;
	if (s->compute)
		ref_compute_fixed(base, s->stride, s->frame_len, cnt,
		                  s->out ? s->out + s->lo : NULL,
		                  s->csums ? s->csums + s->lo : NULL);
	else
		ref_verify_fixed(base, s->stride, s->frame_len, cnt, s->out + s->lo,
		                 s->flags);
	return NULL;
}

static void run_sharded(struct shard proto, uint32_t n, int threads)
{
	enum { MAXT = 256 };
	pthread_t tid[MAXT];
	int live[MAXT];
	struct shard sh[MAXT];
	int t;

	if (threads < 1)
		threads = 1;
	if (threads > MAXT)
		threads = MAXT;
	for (t = 0; t < threads; t++) {
		sh[t] = proto;
		sh[t].lo = (uint32_t)((uint64_t)n * t / threads);
		sh[t].hi = (uint32_t)((uint64_t)n * (t + 1) / threads);
	}
	for (t = 1; t < threads; t++) {
		live[t] = pthread_create(&tid[t], NULL, shard_main, &sh[t]) == 0;
		if (!live[t])
			shard_main(&sh[t]);   /* could not spawn: run the shard inline */
	}
	shard_main(&sh[0]);
	for (t = 1; t < threads; t++)
		if (live[t])
			pthread_join(tid[t], NULL);
}

void ref_verify_fixed_mt(uint8_t *buf, uint64_t stride, uint32_t frame_len,
                         uint32_t n, uint8_t *verdict, uint32_t flags,
                         int threads)
{
	struct shard p = {buf, stride, frame_len, 0, 0, flags, verdict, NULL, 0};
	run_sharded(p, n, threads);
}

void ref_compute_fixed_mt(uint8_t *buf, uint64_t stride, uint32_t frame_len,
                          uint32_t n, uint8_t *status, uint32_t *csums,
                          int threads)
{
	struct shard p = {buf, stride, frame_len, 0, 0, 0, status, csums, 1};
	run_sharded(p, n, threads);
}

void ref_tcp_checksum_batch(const uint8_t *buf, const uint64_t *off,
                            const uint16_t *len, const uint32_t *saddr,
                            const uint32_t *daddr, uint32_t n, uint16_t *out)
{
	uint32_t i;
	for (i = 0; i < n; i++)
		out[i] = ref_tcp_calc_checksum(buf + off[i], len[i], saddr[i], daddr[i]);
}

void ref_ip_checksum_batch(const uint8_t *buf, const uint64_t *off,
                           const uint8_t *ihl, uint32_t n, uint16_t *out)
{
	uint32_t i;
	for (i = 0; i < n; i++)
		out[i] = ref_ip_fast_csum(buf + off[i], ihl[i]);
}

void ref_icmp_checksum_batch(const uint8_t *buf, const uint64_t *off,
                             const uint16_t *len, uint32_t n, uint16_t *out)
{
	uint32_t i;
	for (i = 0; i < n; i++)
		out[i] = ref_icmp_checksum(buf + off[i], len[i]);
}
