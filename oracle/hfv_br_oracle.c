/*
 * hfv_br_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference XDP border router's per-packet path (config 4):
 * border_router/process_packet (br/src/bpf/xdp.c:54-284), parse_underlay/parse_scion/
 * parse_scion_path (br/src/bpf/parser.h:45-204), scion_as_ingress/egress and
 * defer_verify_hop_field (br/src/bpf/path_processing.h:39-152), the fib_lookup_* callers
 * (br/src/bpf/fib_lookup.h:29-261) against the static next-hop table of struct
 * hfv_br_config, and rewrite/rewrite_scion_path (br/src/bpf/rewrite.h:35-146).
 *
 * It works on byte offsets instead of BPF header pointers but keeps the reference's control
 * flow and arithmetic exactly, including its quirks:
 *   - SC_GET_DL/SL mask with 0x2 (scion.h:49-52), so only bit 1 of DL/SL is honoured;
 *   - seg_end adds seg0 for every info field index (path_processing.h:84-86);
 *   - VERDICT_ABORT (XDP action 0) and the bare "return false" of xdp.c:188 are not > 0, so
 *     the packet falls through to the MAC check and the redirect (xdp.c:256-283) and gets a
 *     second record_verdict;
 *   - rewrite happens before verification (xdp.c:242 vs 264);
 *   - the egress HF check uses the current (not switched-to) info field (path_processing.h:142);
 *   - the checksum residuals are u64 sums of little-endian loads of network-order fields and
 *     FOLD_CHECKSUM is applied to ~check + residual + 1 (rewrite.h:35-40, 61-65, 103-106);
 *   - an unknown bpf_fib_lookup return code is treated as success (fib_lookup.h:100-114).
 * One deviation, shared with the GPU kernel: the per-CPU scratchpad is zeroed per packet,
 * so seg_id[1] is 0 when parse_scion_path does not set it (in XDP it holds whatever the
 * previous packet on that CPU left there).
 */
#include <string.h>

#include "../include/scion_hfv.h"
#include "hfv_oracle.h"

enum { A_ABORTED = 0, A_DROP = 1, A_PASS = 2, A_TX = 3, A_REDIRECT = 4 };
#define VERD(action, counter) (((action) & 7) | ((counter) << 3))
enum {
    V_ABORT = VERD(A_ABORTED, 0), V_FORWARD = VERD(A_REDIRECT, 1), V_PARSE_ERROR = VERD(A_DROP, 2),
    V_NOT_SCION = VERD(A_PASS, 3), V_NOT_IMPLEMENTED = VERD(A_PASS, 4), V_NO_INTERFACE = VERD(A_DROP, 5),
    V_UNDERLAY_MISMATCH = VERD(A_PASS, 6), V_ROUTER_ALERT = VERD(A_PASS, 7), V_FIB_DROP = VERD(A_DROP, 8),
    V_FIB_PASS = VERD(A_PASS, 9), V_INVALID_HF = VERD(A_DROP, 10)
};

typedef struct {
    /* packet */
    uint8_t *p;
    long len;
    uint32_t ingress_ifindex;
    const struct hfv_br_config *cfg;
    const orc_hop_key *key;
    uint64_t *stats;
    int last_verdict;
    /* header offsets (struct headers) */
    long eth, ip, udp, scion, meta, inf, hf;
    /* scratchpad (common.h:154-225), zeroed per packet */
    uint32_t verdict;
    uint8_t eth_dst[6], eth_src[6];
    uint32_t family;
    uint32_t v4_dst, v4_src;
    uint8_t v4_ttl;
    uint32_t v6_dst[4], v6_src[4];
    uint8_t v6_hop;
    uint16_t udp_dst, udp_src;
    uint32_t path_type;
    uint32_t feat_off;   /* ORC_BR_NO_*: the build options switched off */
    uint32_t h_meta, curr_inf, curr_hf;
    uint16_t seg_id[2];
    uint32_t segment_switch, seg0, seg1, seg2, num_inf, num_hf;
    uint64_t ip_residual, udp_residual;
    int egress_ifindex;
    uint32_t mask;
    uint8_t macinput[2][16];
    uint64_t mac[2];
} pkt_t;

/* little-endian loads/stores of raw (network-order) fields, as the BPF code does */
static uint16_t l16(const uint8_t *q) { return (uint16_t)(q[0] | q[1] << 8); }
static uint32_t l32(const uint8_t *q) { return (uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16 | (uint32_t)q[3] << 24; }
static void s16(uint8_t *q, uint16_t v) { q[0] = (uint8_t)v; q[1] = (uint8_t)(v >> 8); }
static void s32(uint8_t *q, uint32_t v) { q[0] = (uint8_t)v; q[1] = (uint8_t)(v >> 8); q[2] = (uint8_t)(v >> 16); q[3] = (uint8_t)(v >> 24); }
static uint16_t sw16(uint16_t v) { return (uint16_t)(v << 8 | v >> 8); }
static uint32_t sw32(uint32_t v) { return (v >> 24) | ((v >> 8) & 0xff00) | ((v << 8) & 0xff0000) | (v << 24); }

/* record_verdict (xdp.c:54-70) */
static int record(pkt_t *k, int verdict)
{
    unsigned idx = ((unsigned)verdict >> 3) & 0x0f;
    k->last_verdict = verdict;
    if (k->stats && k->ingress_ifindex < HFV_BR_STATS_IFINDEX && idx < HFV_BR_COUNTERS) {
        uint64_t *row = k->stats + (size_t)k->ingress_ifindex * 2 * HFV_BR_COUNTERS;
        row[idx] += (uint64_t)k->len;
        row[HFV_BR_COUNTERS + idx] += 1;
    }
    return verdict & 0x07;
}

/* ---- parser.h ---------------------------------------------------------------------- */
static long parse_underlay(pkt_t *k, long off)
{
    k->verdict = V_NOT_SCION;
    k->eth = off;
    off += 14;
    if (off > k->len) return -1;
    memcpy(k->eth_dst, k->p + k->eth, 6);
    memcpy(k->eth_src, k->p + k->eth + 6, 6);
    uint16_t proto = l16(k->p + k->eth + 12);
    /* ENABLE_IPV4 / ENABLE_IPV6 off (br/CMakeLists.txt:5-6): that case of the switch is compiled
     * out (parser.h:60, 81), so the frame falls to `default` -- NOT_SCION, XDP_PASS */
    if (proto == sw16(0x0800) && !(k->feat_off & ORC_BR_NO_IPV4)) {
        k->ip = off;
        off += 20;
        if (off > k->len) return -1;
        const uint8_t *ip = k->p + k->ip;
        k->family = HFV_AF_INET;
        k->ip_residual -= (k->v4_dst = l32(ip + 16));
        k->ip_residual -= (k->v4_src = l32(ip + 12));
        k->udp_residual = k->ip_residual;
        k->ip_residual -= (k->v4_ttl = ip[8]);
        size_t skip = 4 * (size_t)(ip[0] & 0x0f) - 20;
        if (skip > 40) return -1;
        off += (long)skip;
        memset(k->v6_dst, 0, sizeof k->v6_dst);
        memset(k->v6_src, 0, sizeof k->v6_src);
        k->v6_hop = 0;
        if (ip[9] != 17) return -1;
    } else if (proto == sw16(0x86DD) && !(k->feat_off & ORC_BR_NO_IPV6)) {
        k->ip = off;
        off += 40;
        if (off > k->len) return -1;
        const uint8_t *ip = k->p + k->ip;
        k->family = HFV_AF_INET6;
        for (int i = 0; i < 4; ++i) {
            k->v6_dst[i] = l32(ip + 24 + 4 * i);
            k->udp_residual -= k->v6_dst[i];
            k->v6_src[i] = l32(ip + 8 + 4 * i);
            k->udp_residual -= k->v6_src[i];
        }
        k->v6_hop = ip[7];
        k->v4_dst = k->v4_src = 0;
        k->v4_ttl = 0;
        if (ip[6] != 17) return -1;
    } else {
        return -1;
    }
    k->udp = off;
    off += 8;
    if (off > k->len) return -1;
    k->udp_residual -= (k->udp_dst = l16(k->p + k->udp + 2));
    k->udp_residual -= (k->udp_src = l16(k->p + k->udp));
    return off;
}

static long parse_scion_path(pkt_t *k, long off)
{
    k->verdict = V_PARSE_ERROR;
    k->meta = off;
    off += 4;
    if (off > k->len) return -1;
    k->udp_residual -= l32(k->p + k->meta);
    k->h_meta = sw32(l32(k->p + k->meta));
    k->seg0 = (k->h_meta >> 12) & 0x3f;
    k->seg1 = (k->h_meta >> 6) & 0x3f;
    k->seg2 = k->h_meta & 0x3f;
    k->num_inf = (k->seg0 > 0) + (k->seg1 > 0) + (k->seg2 > 0);
    k->num_hf = k->seg0 + k->seg1 + k->seg2;
    k->curr_inf = (k->h_meta >> 30) & 0x03;
    k->curr_hf = (k->h_meta >> 24) & 0x3f;
    k->segment_switch = 0;
    long inf = off + (long)k->curr_inf * 8;
    k->inf = inf;
    if (inf + 8 > k->len) return -1;
    k->seg_id[0] = l16(k->p + inf + 2);
    k->udp_residual -= k->seg_id[0];
    if (k->curr_inf + 1 < k->num_inf) {
        inf += 8;
        if (inf + 8 > k->len) return -1;
        k->seg_id[1] = l16(k->p + inf + 2);
    }
    k->hf = off + (long)k->num_inf * 8 + (long)k->curr_hf * 12;
    if (k->hf + 12 > k->len) return -1;
    return off;
}

static long parse_scion(pkt_t *k, long off)
{
    k->verdict = V_PARSE_ERROR;
    k->scion = off;
    off += 28;
    if (off > k->len) return -1;
    const uint8_t *sc = k->p + k->scion;
    if ((sc[0] >> 4) != 0) {
        k->verdict = V_NOT_IMPLEMENTED;
        return -1;
    }
    uint8_t haddr = sc[9];
    off += 8 + 4 * ((haddr >> 2) & 0x2) + 4 * ((haddr >> 6) & 0x2);
    if (off > k->len) return -1;
    k->path_type = sc[8];
    /* ENABLE_SCION_PATH off (br/CMakeLists.txt:7): no case for the standard path (parser.h:140) */
    if (k->path_type == 1 && !(k->feat_off & ORC_BR_NO_SCION_PATH)) return parse_scion_path(k, off);
    k->verdict = V_NOT_IMPLEMENTED;
    return -1;
}

/* ---- path_processing.h ----------------------------------------------------------------- */
static int cons(const pkt_t *k, long inf) { return k->p[inf] & 0x01; }

static void defer_verify(pkt_t *k, int which, long inf, long hf, uint16_t beta_nbo)
{
    k->mask |= 1u << which;
    uint8_t *mi = k->macinput[which];
    memset(mi, 0, 16);
    s16(mi + 2, beta_nbo);
    memcpy(mi + 4, k->p + inf + 4, 4);
    mi[9] = k->p[hf + 1];
    memcpy(mi + 10, k->p + hf + 2, 4);
    k->mac[which] = 0;
    for (int i = 0; i < 6; ++i) k->mac[which] |= (uint64_t)k->p[hf + 6 + i] << (8 * i);
}

static int as_ingress(pkt_t *k)
{
    const uint8_t *hf = k->p + k->hf;
    if (hf[0] & 0x03) {
        k->verdict = V_ROUTER_ALERT;
        return 0;
    }
    uint16_t beta = sw16(k->seg_id[0]);
    if (!cons(k, k->inf)) beta ^= (uint16_t)(hf[7] | hf[6] << 8);
    defer_verify(k, 0, k->inf, k->hf, sw16(beta));
    if (!cons(k, k->inf)) k->seg_id[0] = sw16(beta);
    uint32_t seg_end = k->seg0;
    if (k->curr_inf >= 1) seg_end += k->seg0;
    if (k->curr_inf >= 2) seg_end += k->seg0;
    uint32_t next_hf = k->curr_hf + 1;
    if (next_hf >= k->num_hf) {
        k->verdict = V_NOT_IMPLEMENTED;
        return 0;
    }
    if (next_hf < k->num_hf && next_hf == seg_end) {
        k->segment_switch = 1;
        ++k->curr_inf;
        ++k->curr_hf;
        k->hf += 12;
        if (k->hf + 12 > k->len) {
            k->verdict = V_PARSE_ERROR;
            return 0;
        }
    }
    return 1;
}

static int as_egress(pkt_t *k, uint32_t as_ing_ifid)
{
    k->verdict = A_ABORTED;
    const uint8_t *hf = k->p + k->hf;
    if (hf[0] & 0x03) {
        k->verdict = V_ROUTER_ALERT;
        return 0;
    }
    long inf = k->inf;
    if (k->segment_switch) {
        inf += 8;
        if (inf + 8 > k->len) return 0;
    }
    uint16_t *sid = k->segment_switch ? &k->seg_id[1] : &k->seg_id[0];
    uint16_t beta = sw16(*sid);
    if (as_ing_ifid == 0) defer_verify(k, 1, k->inf, k->hf, sw16(beta));
    if (cons(k, inf)) *sid = sw16((uint16_t)(beta ^ (uint16_t)(hf[7] | hf[6] << 8)));
    ++k->curr_hf;
    return 1;
}

/* ---- tables ------------------------------------------------------------------------------ */
static const struct hfv_br_int_iface *int_iface(const pkt_t *k, uint32_t ifindex)
{
    for (uint32_t i = 0; i < k->cfg->n_int_ifaces && i < HFV_BR_MAX_IFACES; ++i)
        if (k->cfg->int_ifaces[i].ifindex == ifindex) return &k->cfg->int_ifaces[i];
    return NULL;
}

static void addr_bytes(const pkt_t *k, int dst, uint8_t out[16])
{
    memset(out, 0, 16);
    if (k->family == HFV_AF_INET) s32(out, dst ? k->v4_dst : k->v4_src);
    else
        for (int i = 0; i < 4; ++i) s32(out + 4 * i, dst ? k->v6_dst[i] : k->v6_src[i]);
}

/* ingress_map lookup on the struct ingress_addr key {ipv4, ipv6[4], port, u16 ifindex} */
static const struct hfv_br_ingress *ingress_lookup(const pkt_t *k)
{
    uint8_t v4[4], v6[16];
    s32(v4, k->v4_dst);
    for (int i = 0; i < 4; ++i) s32(v6 + 4 * i, k->v6_dst[i]);
    for (uint32_t i = 0; i < k->cfg->n_ingress && i < HFV_BR_MAX_IFACES; ++i) {
        const struct hfv_br_ingress *e = &k->cfg->ingress[i];
        uint8_t e4[4] = {0}, e6[16] = {0};
        if (e->family == HFV_AF_INET) memcpy(e4, e->addr, 4);
        else memcpy(e6, e->addr, 16);
        if (memcmp(e4, v4, 4) == 0 && memcmp(e6, v6, 16) == 0 && l16(e->port) == k->udp_dst &&
            (uint16_t)e->ifindex == (uint16_t)k->ingress_ifindex)
            return e;
    }
    return NULL;
}

static const struct hfv_br_egress *egress_lookup(const pkt_t *k, uint32_t ifid)
{
    for (uint32_t i = 0; i < k->cfg->n_egress && i < HFV_BR_MAX_IFACES; ++i)
        if (k->cfg->egress[i].ifid == ifid) return &k->cfg->egress[i];
    return NULL;
}

/* bpf_fib_lookup replacement: longest prefix match on (family, dst) */
static const struct hfv_br_route *route_lookup(const pkt_t *k, const uint8_t dst[16])
{
    const struct hfv_br_route *best = NULL;
    for (uint32_t i = 0; i < k->cfg->n_routes && i < HFV_BR_MAX_ROUTES; ++i) {
        const struct hfv_br_route *r = &k->cfg->routes[i];
        if (r->family != k->family) continue;
        uint32_t bits = r->prefix_len, maxb = k->family == HFV_AF_INET ? 32 : 128;
        if (bits > maxb) continue;
        int match = 1;
        for (uint32_t b = 0; b < bits; ++b)
            if (((r->prefix[b / 8] ^ dst[b / 8]) >> (7 - b % 8)) & 1) { match = 0; break; }
        if (match && (!best || r->prefix_len > best->prefix_len)) best = r;
    }
    return best;
}

/* result handling shared by the three fib_lookup_* helpers; returns 0 to continue */
static int fib_result(pkt_t *k, const struct hfv_br_route *r)
{
    int ret = r ? r->ret : 4;   /* no route: BPF_FIB_LKUP_RET_NOT_FWDED */
    switch (ret) {
    case 1: case 2: case 3:
        k->verdict = V_FIB_DROP;
        return -1;
    case 4: case 5: case 6: case 7: case 8:
        k->verdict = V_FIB_PASS;
        return -1;
    default:
        break;
    }
    if (r) {
        memcpy(k->eth_dst, r->dmac, 6);
        memcpy(k->eth_src, r->smac, 6);
    } else {
        memset(k->eth_dst, 0, 6);
        memset(k->eth_src, 0, 6);
    }
    return 0;
}

static int fib_as_egress(pkt_t *k, const struct hfv_br_egress *link)
{
    k->udp_dst = l16(link->remote_port);
    k->udp_src = l16(link->local_port);
    if (k->family == HFV_AF_INET) {
        k->v4_dst = l32(link->remote);
        k->v4_src = l32(link->local);
        k->v4_ttl = 64;
    } else if (k->family == HFV_AF_INET6) {
        for (int i = 0; i < 4; ++i) {
            k->v6_dst[i] = l32(link->remote + 4 * i);
            k->v6_src[i] = l32(link->local + 4 * i);
        }
        k->v6_hop = 64;
    }
    const struct hfv_br_route *r = route_lookup(k, link->remote);
    if (fib_result(k, r)) return -1;
    return r ? (int)r->ifindex : 0;
}

static int fib_egress_br(pkt_t *k, const struct hfv_br_egress *sib)
{
    k->udp_dst = l16(sib->remote_port);
    if (k->family == HFV_AF_INET) k->v4_dst = l32(sib->remote);
    else if (k->family == HFV_AF_INET6)
        for (int i = 0; i < 4; ++i) k->v6_dst[i] = l32(sib->remote + 4 * i);
    const struct hfv_br_route *r = route_lookup(k, sib->remote);
    if (fib_result(k, r)) return -1;
    uint32_t out_if = r ? r->ifindex : 0;
    const struct hfv_br_int_iface *src = int_iface(k, out_if);
    if (!src) {
        k->verdict = V_ABORT;
        return -1;
    }
    if (src->family != k->family) {
        k->verdict = V_UNDERLAY_MISMATCH;
        return -1;
    }
    k->udp_src = l16(src->port);
    if (k->family == HFV_AF_INET) {
        k->v4_src = l32(src->addr);
        k->v4_ttl = 64;
    } else if (k->family == HFV_AF_INET6) {
        for (int i = 0; i < 4; ++i) k->v6_src[i] = l32(src->addr + 4 * i);
        k->v6_hop = 64;
    }
    return (int)out_if;
}

static int fib_ip_forward(pkt_t *k)
{
    uint8_t dst[16];
    memset(dst, 0, 16);
    if (k->family == HFV_AF_INET) memcpy(dst, k->p + k->ip + 16, 4);   /* hdr->ip.v4->daddr */
    else addr_bytes(k, 1, dst);
    const struct hfv_br_route *r = route_lookup(k, dst);
    if (fib_result(k, r)) return -1;
    --k->v4_ttl;
    return r ? (int)r->ifindex : 0;
}

/* ---- rewrite.h ----------------------------------------------------------------------------- */
static uint16_t fold(uint64_t c)
{
    c = (c & 0xffff) + (c >> 16);
    c = (c & 0xffff) + (c >> 16);
    c = ~c;
    if (c == 0) c = 0xffff;
    return (uint16_t)c;
}

static void rewrite(pkt_t *k)
{
    memcpy(k->p + k->eth, k->eth_dst, 6);
    memcpy(k->p + k->eth + 6, k->eth_src, 6);
    if (k->family == HFV_AF_INET) {
        uint8_t *ip = k->p + k->ip;
        s32(ip + 16, k->v4_dst);
        s32(ip + 12, k->v4_src);
        uint64_t c = (uint64_t)k->v4_dst + (uint64_t)k->v4_src;
        k->ip_residual += c;
        k->udp_residual += c;
        ip[8] = k->v4_ttl;
        k->ip_residual += k->v4_ttl;
        uint64_t cs = ~(uint64_t)(int64_t)(int32_t)l16(ip + 10) + k->ip_residual + 1;
        s16(ip + 10, fold(cs));
    } else if (k->family == HFV_AF_INET6) {
        uint8_t *ip = k->p + k->ip;
        if (k->ip + 24 + 16 < k->len && k->ip + 8 + 16 < k->len) {
            for (int i = 0; i < 4; ++i) {
                s32(ip + 24 + 4 * i, k->v6_dst[i]);
                k->udp_residual += k->v6_dst[i];
                s32(ip + 8 + 4 * i, k->v6_src[i]);
                k->udp_residual += k->v6_src[i];
            }
        }
        ip[7] = k->v6_hop;
    }
    uint8_t *udp = k->p + k->udp;
    s16(udp + 2, k->udp_dst);
    s16(udp, k->udp_src);
    k->udp_residual += k->udp_dst;
    k->udp_residual += k->udp_src;
    if (k->path_type == 1) {
        uint32_t meta = (k->h_meta & 0x00ffffff) | ((k->curr_hf & 0x3f) << 24) | (k->curr_inf << 30);
        s32(k->p + k->meta, sw32(meta));
        k->udp_residual += sw32(meta);
        long inf = k->inf;
        s16(k->p + inf + 2, k->seg_id[0]);
        k->udp_residual += k->seg_id[0];
        if (k->segment_switch) {
            inf += 8;
            if (inf + 8 <= k->len) {
                k->udp_residual -= l16(k->p + inf + 2);
                k->udp_residual += k->seg_id[1];
                s16(k->p + inf + 2, k->seg_id[1]);
            }
        }
    }
    uint64_t cs = ~(uint64_t)(int64_t)(int32_t)l16(udp + 6) + k->udp_residual + 1;
    s16(udp + 6, fold(cs));
}

/* ---- xdp.c ---------------------------------------------------------------------------------- */
static int process_packet(pkt_t *k)
{
    k->ip_residual = 0;
    k->udp_residual = 0;
    k->egress_ifindex = -1;
    k->mask = 0;
    long off = parse_underlay(k, 0);
    if (off < 0) return record(k, (int)k->verdict);
    off = parse_scion(k, off);
    if (off < 0) return record(k, (int)k->verdict);

    uint32_t as_ing_ifid = 0;
    if (!int_iface(k, k->ingress_ifindex)) {
        const struct hfv_br_ingress *e = ingress_lookup(k);
        if (!e) return record(k, V_NO_INTERFACE);
        as_ing_ifid = e->ifid;
        const uint8_t *hf = k->p + k->hf;
        uint16_t hf_ing = cons(k, k->inf) ? l16(hf + 2) : l16(hf + 4);
        if (sw16(hf_ing) != as_ing_ifid) return record(k, V_NO_INTERFACE);
    }
    if (as_ing_ifid != 0 && k->path_type == 1)
        if (!as_ingress(k)) return record(k, (int)k->verdict);

    long inf = k->inf;
    if (k->segment_switch) {
        inf += 8;
        if (inf + 8 > k->len) return 0;
    }
    const uint8_t *hf = k->p + k->hf;
    uint32_t key = sw16(cons(k, inf) ? l16(hf + 4) : l16(hf + 2));
    const struct hfv_br_egress *fwd = egress_lookup(k, key);
    if (!fwd) return record(k, V_ABORT);

    int egress = -1;
    if (fwd->fwd_external) {
        if (k->path_type == 1)
            if (!as_egress(k, as_ing_ifid)) return record(k, (int)k->verdict);
        if (fwd->family != k->family) return record(k, V_UNDERLAY_MISMATCH);
        egress = fib_as_egress(k, fwd);
    } else if (as_ing_ifid != 0) {
        if (fwd->family != k->family) return record(k, V_UNDERLAY_MISMATCH);
        egress = fib_egress_br(k, fwd);
    } else {
        egress = fib_ip_forward(k);
    }
    if (egress < 0) return record(k, (int)k->verdict);
    rewrite(k);
    k->egress_ifindex = egress;
    return -1;
}

static int tx_port(const struct hfv_br_config *cfg, int ifindex)
{
    if (ifindex < 0 || ifindex >= HFV_BR_MAX_TXPORTS) return 0;
    for (uint32_t i = 0; i < cfg->n_tx_ports && i < HFV_BR_MAX_TXPORTS; ++i)
        if (cfg->tx_ports[i] == (uint32_t)ifindex) return 1;
    return 0;
}

/* border_router, xdp.c:250-283.  hf_check = 0 is the ENABLE_HF_CHECK=OFF build
 * (br/CMakeLists.txt:8,48-64): defer_verify_hop_field and the MAC block compile to nothing
 * (path_processing.h:43-57, xdp.c:259-274), everything else is unchanged. */
static int border_router(pkt_t *k, int hf_check)
{
    int v = process_packet(k);
    if (v > 0) return v;
    for (int w = 0; hf_check && w < 2; ++w) {
        if (!(k->mask & (1u << w))) continue;
        if (!orc_verify_hop_field(k->macinput[w], k->mac[w], k->key)) return record(k, V_INVALID_HF);
    }
    int verdict = A_ABORTED;
    if (tx_port(k->cfg, k->egress_ifindex)) verdict = V_FORWARD;
    return record(k, verdict);
}

void orc_br_process_feat(uint8_t *pkts, size_t slot, const uint16_t *len, const uint32_t *ingress_ifindex, size_t n,
                         const void *cfg, const orc_hop_key *key0, uint8_t *action, uint8_t *verdict,
                         int32_t *egress_ifindex, uint64_t *stats, int hf_check, uint32_t feat_off)
{
    for (size_t i = 0; i < n; ++i) {
        pkt_t k;
        memset(&k, 0, sizeof k);
        k.p = pkts + i * slot;
        k.len = len[i] <= slot ? len[i] : (long)slot;
        k.ingress_ifindex = ingress_ifindex[i];
        k.cfg = (const struct hfv_br_config *)cfg;
        k.key = key0;
        k.stats = stats;
        k.last_verdict = 0;
        k.feat_off = feat_off;
        int a = border_router(&k, hf_check);
        action[i] = (uint8_t)a;
        verdict[i] = (uint8_t)k.last_verdict;
        egress_ifindex[i] = k.egress_ifindex;
    }
}

void orc_br_process_ex(uint8_t *pkts, size_t slot, const uint16_t *len, const uint32_t *ingress_ifindex, size_t n,
                       const void *cfg, const orc_hop_key *key0, uint8_t *action, uint8_t *verdict,
                       int32_t *egress_ifindex, uint64_t *stats, int hf_check)
{
    orc_br_process_feat(pkts, slot, len, ingress_ifindex, n, cfg, key0, action, verdict, egress_ifindex, stats, hf_check,
                        0);
}

void orc_br_process(uint8_t *pkts, size_t slot, const uint16_t *len, const uint32_t *ingress_ifindex, size_t n,
                    const void *cfg, const orc_hop_key *key0, uint8_t *action, uint8_t *verdict,
                    int32_t *egress_ifindex, uint64_t *stats)
{
    orc_br_process_ex(pkts, slot, len, ingress_ifindex, n, cfg, key0, action, verdict, egress_ifindex, stats, 1);
}
