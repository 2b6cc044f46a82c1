// hfv_br_kernel.hip -- the reference XDP border router's whole per-packet path (config 4) on
// gfx950: parse Ethernet/IPv4|IPv6/UDP/SCION, AS ingress/egress hop processing, next-hop
// lookup, in-place rewrite with incremental checksums, deferred hop-field AES-CMAC check,
// redirect decision and verdict counters.
//
// Follows, function by function:
//   border_router / process_packet / record_verdict / verify_hop_field  br/src/bpf/xdp.c:54-284
//   parse_underlay / parse_scion / parse_scion_path                      br/src/bpf/parser.h:45-204
//   defer_verify_hop_field / scion_as_ingress / scion_as_egress          br/src/bpf/path_processing.h:39-152
//   fib_lookup_as_egress / fib_lookup_egress_br / fib_lookup_ip_forward  br/src/bpf/fib_lookup.h:29-261
//   rewrite / rewrite_scion_path                                         br/src/bpf/rewrite.h:35-146
// with the reference's quirks kept (listed in oracle/hfv_br_oracle.c, the CPU checker).
// bpf_fib_lookup is replaced by the static next-hop table of the installed hfv_br_config.
//
// Mapping: one lane per frame, a persistent grid with one block per CU (1024 threads = 16 waves).
// Each block builds the AES round tables in LDS (T0/T1, 8 lane replicas, 16 KiB: AES is a small
// part of the router's work, so LDS goes to header rows),
// and stages the router tables (~6.5 KiB), its verdict counters (5.5 KiB of 32-bit words) and, in
// the staged variant, the first 128 bytes of each frame of its waves' tiles (a frame whose header
// runs past them also gets bytes 128-135 in registers, HFV_BR_EXT).  The rewrite patches the
// staged rows, and only the 16-byte chunks it touched go back to HBM; payload bytes are never
// read.  At most one hop field is checked per frame (ingress from a neighbour AS or
// egress of a packet from the own AS), with the record-verify kernel's AES code (slot-0 key
// in SGPRs).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdlib.h>

// Staging waves per CU: 16 (AES tables with 4 lane copies, to fit the 16 header-row buffers in
// LDS; VGPRs capped at 128, which the frame state fits since the rewrite reads its inputs from
// the staged row and the tables: 124, no scratch) or 12 (16 copies; 14 % slower).
#ifndef HFV_BR_WAVES
#define HFV_BR_WAVES 16
#endif
// HFV_BR_STATS32 = 1: the block's verdict counters in 32-bit LDS words (5.5 KiB instead of 11),
// added into the caller's 64-bit counters at the end of the launch; launch_br_process splits a
// launch so that no block can count 2^32 bytes.  The LDS this frees holds 8 lane copies of the
// AES tables instead of 4.
#ifndef HFV_BR_STATS32
#define HFV_BR_STATS32 1
#endif
#ifndef HFV_TAB3_COPIES
#if HFV_BR_WAVES == 16 && HFV_BR_STATS32
#define HFV_TAB3_COPIES 8
#elif HFV_BR_WAVES == 16
#define HFV_TAB3_COPIES 4
#else
#define HFV_TAB3_COPIES 16
#endif
#endif
#include "hfv_aes_dev.h"
#include "hfv_internal.h"

namespace hfv {

static __shared__ DevBrConfig s_br;
#if HFV_BR_STATS32
typedef uint32_t BrCount;
#else
typedef unsigned long long BrCount;
#endif
static __shared__ BrCount s_stats[HFV_BR_STATS_IFINDEX * 2 * HFV_BR_COUNTERS];

// Header staging (WIN > 0 kernels): the first kBrWin bytes of each frame of a wave's 64-frame
// tile, one row of kBrWin / 4 + 1 dwords per frame (the odd row pitch keeps both the staging
// writes and the per-lane reads bank-conflict free), for up to kBrStageWaves waves per block.
constexpr int kBrWin = 128;
constexpr int kBrRow = kBrWin / 4 + 1;
constexpr int kBrStageWaves = HFV_BR_WAVES;
static __shared__ uint32_t s_hdr[kBrStageWaves * 64 * kBrRow];

// HFV_BR_PROF = 1: diagnostic build.  Each wave adds the shader cycles (s_memtime) it spends in
// the phases of a tile into g_br_prof (read by hfv_debug_br_prof): [0] header loads issued ->
// staged, [1] parse/process_packet, [2] MAC check + outputs, [3] write-back, [4] tiles.
#ifndef HFV_BR_PROF
#define HFV_BR_PROF 0
#endif
// HFV_BR_WB: order of a tile's write-back against the next tile's header loads.
//   0: stores, then the next tile's loads at the top of the loop (vmcnt retires in order, so
//      the wait for the loads also waits for the stores' acknowledgement);
//   1: the changed chunks are read from LDS into registers, the next tile's loads are issued,
//      then the chunks go out as buffer stores whose lanes without a change address past the
//      tile's buffer range (dropped by the bounds check: no branch, a fixed count of stores), and
//      the loop waits for the loads only (vmcnt = that count);
//   9: diagnostic, no write-back at all (wrong output: measures what the stores cost).
#ifndef HFV_BR_WB
#define HFV_BR_WB 1
#endif
// HFV_BR_DYN (with HFV_BR_WB == 1): 1 = each block owns a contiguous tile range and its waves
// claim the next tile from a block-local LDS counter at the end of the current one, so a wave
// that ran fast takes more; 0 = tile t goes to wave (t mod waves) statically.
#ifndef HFV_BR_DYN
#define HFV_BR_DYN 1
#endif
static __shared__ uint32_t s_br_next;
#if HFV_BR_PROF
__device__ unsigned long long g_br_prof[8];
#endif
struct BrProf {
    uint64_t c[5] = {0, 0, 0, 0, 0};
    uint64_t t = 0;
    __device__ __forceinline__ void start()
    {
        if constexpr (HFV_BR_PROF) t = __builtin_amdgcn_s_memtime();
    }
    __device__ __forceinline__ void mark(int i)
    {
        if constexpr (HFV_BR_PROF) {
            const uint64_t x = __builtin_amdgcn_s_memtime();
            c[i] += x - t;
            t = x;
        }
    }
};

// enum xdp_action and enum verdict (br/src/bpf/common.h:38-70)
enum : uint32_t { A_ABORTED = 0, A_DROP = 1, A_PASS = 2, A_TX = 3, A_REDIRECT = 4 };
constexpr uint32_t verd(uint32_t action, uint32_t counter) { return (action & 7u) | (counter << 3); }
enum : uint32_t {
    V_ABORT = verd(A_ABORTED, 0), V_FORWARD = verd(A_REDIRECT, 1), V_PARSE_ERROR = verd(A_DROP, 2),
    V_NOT_SCION = verd(A_PASS, 3), V_NOT_IMPLEMENTED = verd(A_PASS, 4), V_NO_INTERFACE = verd(A_DROP, 5),
    V_UNDERLAY_MISMATCH = verd(A_PASS, 6), V_ROUTER_ALERT = verd(A_PASS, 7), V_FIB_DROP = verd(A_DROP, 8),
    V_FIB_PASS = verd(A_PASS, 9), V_INVALID_HF = verd(A_DROP, 10)
};

// The BPF code reads and writes network-order fields through little-endian u16/u32 views.
__device__ __forceinline__ uint32_t g8(const uint8_t *q) { return q[0]; }
__device__ __forceinline__ uint32_t g16(const uint8_t *q) { return (uint32_t)q[0] | ((uint32_t)q[1] << 8); }
__device__ __forceinline__ uint32_t g32(const uint8_t *q)
{
    return (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
}
__device__ __forceinline__ uint32_t sw16(uint32_t v) { return ((v & 0xffu) << 8) | ((v >> 8) & 0xffu); }
__device__ __forceinline__ uint32_t sw32(uint32_t v) { return __builtin_bswap32(v); }

// Per-frame state: struct headers + the per-CPU scratchpad (common.h:154-225), zeroed per frame.
struct BrFrame {
    const uint8_t *p;   // the frame as received (reads past the window)
    uint8_t *po;        // where its changed bytes go (p itself, or the caller's output copy)
    uint32_t row;      // dword index of this frame's staged header row in s_hdr
    int win;           // staged bytes (0: read and write everything in HBM)
    // bytes win..win+7, loaded into registers at the start of the frame when its SCION header
    // (HdrLen) runs past the window (HFV_BR_EXT): one early load instead of a round trip per field
    uint32_t ext[2];
    bool has_ext;
    uint32_t dirty;    // 16-byte chunks of the staged row written (only those go back to HBM)
    int len;
    int lim;           // bytes of the frame present in the buffer (min(len, window))
    bool cut;          // a check failed only because the window ended before len

    uint32_t ifindex;
    uint32_t last_verdict;
    int ip, udp, meta, inf, hf;
    uint32_t verdict;
    uint32_t family;
    uint32_t h_meta, curr_inf, curr_hf;
    uint32_t seg_id0, seg_id1;
    uint32_t segment_switch, seg0, num_inf, num_hf;
    // The next hop, as table indices: the rewrite reads the new addresses, ports and MACs from
    // the LDS tables and the original header fields (and so the checksum residuals of
    // rewrite.h) from the staged row, instead of the frame carrying ~20 registers of them from
    // the parse to the rewrite.  nh: 0 IP forward (fib_lookup_ip), 1 external link, 2 sibling.
    uint32_t nh;
    int fwd, sib_if, route;
    int egress_ifindex;
    // deferred MAC check: ingress (mask bit 0) and egress-from-internal (bit 1) never both apply
    bool need_mac;
    int mac_inf, mac_hf;
    uint32_t mac_beta;
    uint32_t clob;      // bit 0 / 1: the rewrite's SegID store at INF+2 / INF+10 lands in the hop field
    uint32_t orig_ab;   // those bytes before the rewrite (INF+2..3 | INF+10..11 << 16)
};

// Header reads (the BPF code's little-endian loads of network-order fields): bytes inside the
// staged window come from LDS (a 32-bit field = two aligned ds_read_b32 + v_alignbyte), the
// rest from the frame in HBM.  The LDS read is unconditional (clamped into the row) and only
// the rare read past the window is a branch, so reads of independent fields can share one wait
// (1 % faster than the LDS read inside the branch: most of the parse's waits are data-dependent,
// each offset coming from the previous field).
__device__ __forceinline__ uint32_t lds_u32_at(const BrFrame &k, int off)
{
    const uint32_t *row = s_hdr + k.row;
    int a = off >> 2;
    return __builtin_amdgcn_alignbyte(row[a + 1], row[a], (uint32_t)(off & 3));
}
// The wait for a read past the window sits inside its branch: placed after the merge by the
// waitcnt pass, a vmcnt(0) would run on every path and wait for the previous tile's write-back
// stores, which vmcnt retires in order before this read (HFV_BR_WB == 1 leaves them in flight).
__device__ __forceinline__ void wait_past_window() { __builtin_amdgcn_s_waitcnt(0x0F70); }   // vmcnt(0)
// HFV_BR_EXT = 1: frames whose SCION header (by its HdrLen) ends past the window get the next 8
// bytes (the bench mix's longest headers end at 136) with one load issued before the parse; their
// reads of those bytes come from registers.
#ifndef HFV_BR_EXT
#define HFV_BR_EXT 1
#endif
constexpr int kBrExt = 8;
// the 32 bits starting at byte b (0 <= b <= 4, or b <= 6 for the low 16) of the frame's ext bytes
__device__ __forceinline__ uint32_t ext_u32(const BrFrame &k, int b)
{
    return __builtin_amdgcn_alignbyte(k.ext[1], b < 4 ? k.ext[0] : k.ext[1], (uint32_t)b & 3u);
}
__device__ __forceinline__ bool in_ext(const BrFrame &k, int off, int size)
{
    return HFV_BR_EXT && k.has_ext && off >= k.win && off + size <= k.win + kBrExt;
}
__device__ __forceinline__ uint32_t rd8(const BrFrame &k, int off)
{
    if (k.win == 0) return g8(k.p + off);
    const bool in = (uint32_t)off < (uint32_t)k.win;
    uint32_t v = reinterpret_cast<const uint8_t *>(s_hdr + k.row)[in ? off : 0];
    if (!in) {
        if (in_ext(k, off, 1)) {
            v = ext_u32(k, off - k.win) & 0xffu;
        } else {
            v = g8(k.p + off);
            wait_past_window();
        }
    }
    return v;
}
// Every 16- and 32-bit header field sits at an even offset (Ethernet 14 B, IP header lengths in
// 4-byte units, UDP 8, SCION common header 12, host addresses in 4-byte units, info fields 8 and
// hop fields 12 B), so a 16-bit field is one ds_read_u16 / ds_write_b16 of the staged row
// instead of two dword reads + v_alignbyte / two byte stores (round 5: 79.8-80.4 against
// 80.1-80.9 us, profiles/r05/s17/).
__device__ __forceinline__ uint32_t lds_u16_at(const BrFrame &k, int off)
{
    return *reinterpret_cast<const uint16_t *>(reinterpret_cast<const uint8_t *>(s_hdr + k.row) + off);
}
__device__ __forceinline__ uint32_t rd16(const BrFrame &k, int off)
{
    if (k.win == 0) return g16(k.p + off);
    const bool in = (uint32_t)off + 2 <= (uint32_t)k.win;
    uint32_t v = lds_u16_at(k, in ? off : 0);
    if (!in) {
        if (in_ext(k, off, 2)) {
            v = ext_u32(k, off - k.win) & 0xffffu;
        } else {
            v = g16(k.p + off);
            wait_past_window();
        }
    }
    return v;
}
__device__ __forceinline__ uint32_t rd32(const BrFrame &k, int off)
{
    if (k.win == 0) return g32(k.p + off);
    const bool in = (uint32_t)off + 4 <= (uint32_t)k.win;
    uint32_t v = lds_u32_at(k, in ? off : 0);
    if (!in) {
        if (in_ext(k, off, 4)) {
            v = ext_u32(k, off - k.win);
        } else {
            v = g32(k.p + off);
            wait_past_window();
        }
    }
    return v;
}

// Header writes: bytes inside the staged window go to the LDS row (written back to HBM with
// coalesced 16-byte stores at the end of the tile), bytes past it straight to HBM.  As with the
// reads, the LDS store is unconditional: a field not wholly inside the window is stored into
// the row's pad dword (bytes kBrWin..kBrWin+3, never read for a result nor written back) and
// then handled on the rare branch.
constexpr int kBrPad = kBrWin;
__device__ __forceinline__ uint32_t chunk_bit(int off) { return 1u << ((uint32_t)off >> 4 & 31u); }
__device__ __forceinline__ void wr8(BrFrame &k, int off, uint32_t v)
{
    if (k.win == 0) { k.po[off] = (uint8_t)v; return; }
    const bool in = (uint32_t)off < (uint32_t)k.win;
    reinterpret_cast<uint8_t *>(s_hdr + k.row)[in ? off : kBrPad] = (uint8_t)v;
    k.dirty |= in ? chunk_bit(off) : 0u;
    if (!in) k.po[off] = (uint8_t)v;
}
__device__ __forceinline__ void wr16(BrFrame &k, int off, uint32_t v)
{
    if (k.win == 0) { k.po[off] = (uint8_t)v; k.po[off + 1] = (uint8_t)(v >> 8); return; }
    const bool in = (uint32_t)off + 2 <= (uint32_t)k.win;   // whole field in the window (the common case)
    uint8_t *q = reinterpret_cast<uint8_t *>(s_hdr + k.row) + (in ? off : kBrPad);
    *reinterpret_cast<uint16_t *>(q) = (uint16_t)v;
    k.dirty |= in ? chunk_bit(off) | chunk_bit(off + 1) : 0u;
    if (!in) {
        if (off >= k.win) {
            k.po[off] = (uint8_t)v; k.po[off + 1] = (uint8_t)(v >> 8);
        } else {
            wr8(k, off, v);
            wr8(k, off + 1, v >> 8);
        }
    }
}
__device__ __forceinline__ void wr32(BrFrame &k, int off, uint32_t v)
{
    if (k.win == 0) {
        uint8_t *q = k.po + off;
        q[0] = (uint8_t)v; q[1] = (uint8_t)(v >> 8); q[2] = (uint8_t)(v >> 16); q[3] = (uint8_t)(v >> 24);
        return;
    }
    const bool in = (uint32_t)off + 4 <= (uint32_t)k.win;
    uint8_t *q = reinterpret_cast<uint8_t *>(s_hdr + k.row) + (in ? off : kBrPad);
    reinterpret_cast<uint16_t *>(q)[0] = (uint16_t)v;
    reinterpret_cast<uint16_t *>(q)[1] = (uint16_t)(v >> 16);
    k.dirty |= in ? chunk_bit(off) | chunk_bit(off + 3) : 0u;
    if (!in) {
        if (off >= k.win) {
            uint8_t *h = k.po + off;
            h[0] = (uint8_t)v; h[1] = (uint8_t)(v >> 8); h[2] = (uint8_t)(v >> 16); h[3] = (uint8_t)(v >> 24);
        } else {
            wr16(k, off, v);
            wr16(k, off + 2, v >> 16);
        }
    }
}

// Bounds check of the BPF code ("data + n > data_end").  With a header window smaller than the
// frame, running past the window marks the frame `cut` (the host path re-runs it whole).
__device__ __forceinline__ bool beyond(BrFrame &k, int end)
{
    if (end <= k.lim) return false;
    if (end <= k.len) k.cut = true;
    return true;
}

template <bool STATS>
__device__ __forceinline__ uint32_t record(BrFrame &k, uint32_t verdict)   // record_verdict, xdp.c:54-70
{
    uint32_t idx = (verdict >> 3) & 0x0fu;
    k.last_verdict = verdict;
    if constexpr (STATS) {
        if (k.cut) return verdict & 7u;
        if (k.ifindex < HFV_BR_STATS_IFINDEX && idx < HFV_BR_COUNTERS) {
            BrCount *row = s_stats + k.ifindex * 2 * HFV_BR_COUNTERS;
            atomicAdd(row + idx, (BrCount)k.len);
            atomicAdd(row + HFV_BR_COUNTERS + idx, (BrCount)1);
        }
    }
    return verdict & 7u;
}

// ---- parser.h ----------------------------------------------------------------------------
__device__ __forceinline__ int parse_underlay(BrFrame &k)
{
    k.verdict = V_NOT_SCION;
    int off = 14;
    if (beyond(k, off)) return -1;
    uint32_t proto = rd16(k, 12);
    // HFV_BR_NO_IPV4 / _IPV6: the reference built without that case (parser.h:60,81) -> default
    if (proto == 0x0008u && !(s_br.feat_off & HFV_BR_NO_IPV4)) {   // ETH_P_IP, network order
        k.ip = off;
        off += 20;
        if (beyond(k, off)) return -1;
        k.family = HFV_AF_INET;
        int skip = 4 * (int)(rd8(k, k.ip) & 0x0fu) - 20;
        if (skip < 0 || skip > 40) return -1;
        off += skip;
        if (rd8(k, k.ip + 9) != 17u) return -1;
    } else if (proto == 0xdd86u && !(s_br.feat_off & HFV_BR_NO_IPV6)) {   // ETH_P_IPV6
        k.ip = off;
        off += 40;
        if (beyond(k, off)) return -1;
        k.family = HFV_AF_INET6;
        if (rd8(k, k.ip + 6) != 17u) return -1;
    } else {
        return -1;
    }
    k.udp = off;
    off += 8;
    if (beyond(k, off)) return -1;
    return off;
}

__device__ __forceinline__ int parse_scion_path(BrFrame &k, int off)
{
    k.verdict = V_PARSE_ERROR;
    k.meta = off;
    off += 4;
    if (beyond(k, off)) return -1;
    k.h_meta = sw32(rd32(k, k.meta));
    k.seg0 = (k.h_meta >> 12) & 0x3fu;
    uint32_t seg1 = (k.h_meta >> 6) & 0x3fu, seg2 = k.h_meta & 0x3fu;
    k.num_inf = (k.seg0 > 0) + (seg1 > 0) + (seg2 > 0);
    k.num_hf = k.seg0 + seg1 + seg2;
    k.curr_inf = (k.h_meta >> 30) & 0x03u;
    k.curr_hf = (k.h_meta >> 24) & 0x3fu;
    int inf = off + (int)k.curr_inf * 8;
    k.inf = inf;
    if (beyond(k, inf + 8)) return -1;
    k.seg_id0 = rd16(k, inf + 2);
    if (k.curr_inf + 1 < k.num_inf) {
        inf += 8;
        if (beyond(k, inf + 8)) return -1;
        k.seg_id1 = rd16(k, inf + 2);
    }
    k.hf = off + (int)k.num_inf * 8 + (int)k.curr_hf * 12;
    if (beyond(k, k.hf + 12)) return -1;
    return off;
}

__device__ __forceinline__ int parse_scion(BrFrame &k, int off)
{
    k.verdict = V_PARSE_ERROR;
    int sc = off;
    off += 28;
    if (beyond(k, off)) return -1;
    if ((rd8(k, sc) >> 4) != 0) {
        k.verdict = V_NOT_IMPLEMENTED;
        return -1;
    }
    uint32_t haddr = rd8(k, sc + 9);
    off += 8 + 4 * (int)((haddr >> 2) & 0x2u) + 4 * (int)((haddr >> 6) & 0x2u);   // SC_GET_DL/SL, scion.h:49-52
    if (beyond(k, off)) return -1;
    // path_type SCION, unless built without ENABLE_SCION_PATH (parser.h:140)
    if (rd8(k, sc + 8) == 1u && !(s_br.feat_off & HFV_BR_NO_SCION_PATH)) return parse_scion_path(k, off);
    k.verdict = V_NOT_IMPLEMENTED;
    return -1;
}

// ---- path_processing.h ---------------------------------------------------------------------
__device__ __forceinline__ uint32_t cons_at(const BrFrame &k, int inf) { return rd8(k, inf) & 1u; }

// Only the fields' positions are kept: the macinput is read when the MAC is checked, after the
// rewrite (one copy of the reads for the ingress and egress paths of a wave instead of one per
// path).  The rewrite never stores into the timestamp; it stores into the hop field only when
// CurrINF points past the info fields, and keep_mac_bytes saves those bytes first.
__device__ __forceinline__ void defer_verify(BrFrame &k, int inf, int hf, uint32_t beta_nbo)
{
    k.need_mac = true;
    k.mac_inf = inf;
    k.mac_hf = hf;
    k.mac_beta = beta_nbo;
}

__device__ __forceinline__ bool as_ingress(BrFrame &k)
{
    if (rd8(k, k.hf) & 0x03u) {
        k.verdict = V_ROUTER_ALERT;
        return false;
    }
    uint32_t c = cons_at(k, k.inf);
    uint32_t beta = sw16(k.seg_id0);
    if (!c) beta ^= rd8(k, k.hf + 7) | (rd8(k, k.hf + 6) << 8);
    defer_verify(k, k.inf, k.hf, sw16(beta));
    if (!c) k.seg_id0 = sw16(beta);
    uint32_t seg_end = k.seg0;   // path_processing.h:84-86 adds seg0 for every index
    if (k.curr_inf >= 1) seg_end += k.seg0;
    if (k.curr_inf >= 2) seg_end += k.seg0;
    uint32_t next_hf = k.curr_hf + 1;
    if (next_hf >= k.num_hf) {
        k.verdict = V_NOT_IMPLEMENTED;
        return false;
    }
    if (next_hf == seg_end) {
        k.segment_switch = 1;
        ++k.curr_inf;
        ++k.curr_hf;
        k.hf += 12;
        if (beyond(k, k.hf + 12)) {
            k.verdict = V_PARSE_ERROR;
            return false;
        }
    }
    return true;
}

__device__ __forceinline__ bool as_egress(BrFrame &k, uint32_t as_ing_ifid)
{
    k.verdict = A_ABORTED;
    if (rd8(k, k.hf) & 0x03u) {
        k.verdict = V_ROUTER_ALERT;
        return false;
    }
    int inf = k.inf;
    if (k.segment_switch) {
        inf += 8;
        if (beyond(k, inf + 8)) return false;
    }
    uint32_t sid = k.seg_id0;
    if (k.segment_switch) sid = k.seg_id1;
    uint32_t beta = sw16(sid);
    if (as_ing_ifid == 0) defer_verify(k, k.inf, k.hf, sw16(beta));   // original INF, path_processing.h:142
    if (cons_at(k, inf)) {
        uint32_t nb = sw16((beta ^ (rd8(k, k.hf + 7) | (rd8(k, k.hf + 6) << 8))) & 0xffffu);
        if (k.segment_switch) k.seg_id1 = nb;
        else k.seg_id0 = nb;
    }
    ++k.curr_hf;
    return true;
}

// ---- tables (LDS) ----------------------------------------------------------------------------
__device__ __forceinline__ int int_iface(uint32_t ifindex)
{
    if (ifindex < 64) return s_br.int_of_ifindex[ifindex];
    for (uint32_t i = 0; i < s_br.n_int; ++i)
        if (s_br.int_ifaces[i].ifindex == ifindex) return (int)i;
    return -1;
}

// The frame's destination as the ingress_map key holds it (common.h:94-103): the IPv4 address
// with the IPv6 words zero, or the IPv6 words with the IPv4 address zero; and its UDP port.
struct DstKey {
    uint32_t v4, v6[4], port;
};
__device__ __forceinline__ DstKey dst_key(const BrFrame &k)
{
    DstKey d = {};
    if (k.family == HFV_AF_INET) {
        d.v4 = rd32(k, k.ip + 16);
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) d.v6[i] = rd32(k, k.ip + 24 + 4 * i);
    }
    d.port = rd16(k, k.udp + 2);
    return d;
}

__device__ __forceinline__ bool ingress_match(const DevBrIngress &e, const DstKey &d, uint32_t ifindex)
{
    // bitwise, not short-circuit: seven compares of LDS words, no branch (and exec mask) per field
    return (e.v4 == d.v4) & (e.v6[0] == d.v6[0]) & (e.v6[1] == d.v6[1]) & (e.v6[2] == d.v6[2]) & (e.v6[3] == d.v6[3]) &
           (e.port == d.port) & (e.ifindex16 == (ifindex & 0xffffu));
}

__device__ __forceinline__ int ingress_lookup(const BrFrame &k)
{
    const uint32_t x = k.ifindex & 0xffffu;
    int c = -2;
    if (x < 64) {   // the only entry on this interface, if there is just one
        c = s_br.ing_of_ifindex[x];
        if (c == -1) return -1;
    }
    const DstKey d = dst_key(k);
    if (c >= 0) return ingress_match(s_br.ingress[c], d, k.ifindex) ? c : -1;
    for (uint32_t i = 0; i < s_br.n_ing; ++i)
        if (ingress_match(s_br.ingress[i], d, k.ifindex)) return (int)i;
    return -1;
}

__device__ __forceinline__ int egress_lookup(uint32_t ifid)
{
    if (ifid < 256) return s_br.egr_of_ifid[ifid];
    for (uint32_t i = 0; i < s_br.n_egr; ++i)
        if (s_br.egress[i].ifid == ifid) return (int)i;
    return -1;
}

// longest-prefix match on (family, destination as big-endian words); ties keep the first entry
__device__ __forceinline__ int route_lookup(uint32_t family, uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3)
{
    int best = -1;
    uint32_t best_len = 0;
    for (uint32_t i = 0; i < s_br.n_routes; ++i) {
        const DevBrRoute &r = s_br.routes[i];
        if (r.family != family) continue;
        uint32_t diff = ((d0 ^ r.pfx[0]) & r.mask[0]) | ((d1 ^ r.pfx[1]) & r.mask[1]) | ((d2 ^ r.pfx[2]) & r.mask[2]) |
                        ((d3 ^ r.pfx[3]) & r.mask[3]);
        if (diff == 0 && (best < 0 || r.plen > best_len)) {
            best = (int)i;
            best_len = r.plen;
        }
    }
    return best;
}

// bpf_fib_lookup return-code handling shared by the fib_lookup_* helpers; false = stop.  The
// route's MAC addresses are read by the rewrite (k.route).
__device__ __forceinline__ bool fib_result(BrFrame &k, int r)
{
    int ret = r >= 0 ? s_br.routes[r].ret : 4;   // no route: BPF_FIB_LKUP_RET_NOT_FWDED
    if (ret >= 1 && ret <= 3) {
        k.verdict = V_FIB_DROP;
        return false;
    }
    if (ret >= 4 && ret <= 8) {
        k.verdict = V_FIB_PASS;
        return false;
    }
    k.route = r;
    return true;
}

// fib_lookup_ip's route: hdr->ip.v4->daddr or the IPv6 destination
__device__ __forceinline__ int ip_route(const BrFrame &k)
{
    if (k.family == HFV_AF_INET) return route_lookup(k.family, sw32(rd32(k, k.ip + 16)), 0, 0, 0);
    return route_lookup(k.family, sw32(rd32(k, k.ip + 24)), sw32(rd32(k, k.ip + 28)), sw32(rd32(k, k.ip + 32)),
                        sw32(rd32(k, k.ip + 36)));
}

// ---- rewrite.h -------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t fold_checksum(uint64_t c)
{
    c = (c & 0xffffu) + (c >> 16);
    c = (c & 0xffffu) + (c >> 16);
    c = ~c;
    if (c == 0) c = 0xffff;
    return (uint32_t)(c & 0xffffu);
}

// rewrite / rewrite_scion_path (rewrite.h:35-146).  The BPF code subtracts every original
// field from its u64 checksum residuals as it parses them and adds the new values here; the
// residuals are sums mod 2^64, so taking the originals from the staged row (nothing is written
// before they are read) and both sums here gives the same residuals.  New values: the route's
// MACs; for a link (nh 1) or a sibling (nh 2) the link's remote address and port as the
// destination and the link's local (or the sibling's internal interface's) address and port
// as the source with TTL / hop limit 64; for an IP forward (nh 0) the original addresses and
// ports and the IPv4 TTL decremented.
__device__ __forceinline__ void rewrite(BrFrame &k)
{
    const bool fw = k.nh != 0;
    const DevBrEgress &e = s_br.egress[fw ? k.fwd : 0];
    const DevBrIntIface &si = s_br.int_ifaces[k.nh == 2 ? k.sib_if : 0];
    const bool sib = k.nh == 2;
    const uint32_t od_port = rd16(k, k.udp + 2), os_port = rd16(k, k.udp);
    const uint32_t o_seg0 = rd16(k, k.inf + 2);
    uint64_t udp_res = 0;
    udp_res -= (uint64_t)od_port;
    udp_res -= (uint64_t)os_port;
    udp_res -= (uint64_t)sw32(k.h_meta);
    udp_res -= (uint64_t)o_seg0;
    {
        const DevBrRoute &rt = s_br.routes[k.route >= 0 ? k.route : 0];
        const bool ok = k.route >= 0;
        wr32(k, 0, ok ? rt.dmac_lo : 0u); wr16(k, 4, ok ? rt.dmac_hi : 0u);
        wr32(k, 6, ok ? rt.smac_lo : 0u); wr16(k, 10, ok ? rt.smac_hi : 0u);
    }
    if (k.family == HFV_AF_INET) {
        const uint32_t od = rd32(k, k.ip + 16), os = rd32(k, k.ip + 12), ottl = rd8(k, k.ip + 8);
        const uint32_t nd = fw ? e.remote[0] : od;
        const uint32_t ns = fw ? (sib ? si.addr[0] : e.local[0]) : os;
        const uint32_t nttl = fw ? 64u : ((ottl - 1u) & 0xffu);
        const uint64_t c = (uint64_t)nd + (uint64_t)ns - (uint64_t)od - (uint64_t)os;
        wr32(k, k.ip + 16, nd);
        wr32(k, k.ip + 12, ns);
        udp_res += c;
        wr8(k, k.ip + 8, nttl);
        const uint64_t ip_res = c + (uint64_t)nttl - (uint64_t)ottl;
        uint64_t cs = ~(uint64_t)rd16(k, k.ip + 10) + ip_res + 1;
        wr16(k, k.ip + 10, fold_checksum(cs));
    } else {
        const bool put = k.ip + 24 + 16 < k.len && k.ip + 8 + 16 < k.len;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t od = rd32(k, k.ip + 24 + 4 * i), os = rd32(k, k.ip + 8 + 4 * i);
            udp_res -= (uint64_t)od;
            udp_res -= (uint64_t)os;
            if (put) {
                const uint32_t nd = fw ? e.remote[i] : od;
                const uint32_t ns = fw ? (sib ? si.addr[i] : e.local[i]) : os;
                wr32(k, k.ip + 24 + 4 * i, nd);
                wr32(k, k.ip + 8 + 4 * i, ns);
                udp_res += (uint64_t)nd;
                udp_res += (uint64_t)ns;
            }
        }
        if (fw) wr8(k, k.ip + 7, 64u);
        else wr8(k, k.ip + 7, rd8(k, k.ip + 7));   // the BPF code stores the unchanged hop limit
    }
    const uint32_t nd_port = fw ? e.remote_port : od_port;
    const uint32_t ns_port = fw ? (sib ? si.port : e.local_port) : os_port;
    wr16(k, k.udp + 2, nd_port);
    wr16(k, k.udp, ns_port);
    udp_res += (uint64_t)nd_port;
    udp_res += (uint64_t)ns_port;
    // path_type is SCION here (the only type process_packet lets through)
    uint32_t meta = (k.h_meta & 0x00ffffffu) | ((k.curr_hf & 0x3fu) << 24) | (k.curr_inf << 30);
    wr32(k, k.meta, sw32(meta));
    udp_res += (uint64_t)sw32(meta);
    int inf = k.inf;
    wr16(k, inf + 2, k.seg_id0);
    udp_res += (uint64_t)k.seg_id0;
    if (k.segment_switch) {
        inf += 8;
        if (inf + 8 <= k.len) {
            udp_res -= (uint64_t)rd16(k, inf + 2);
            udp_res += (uint64_t)k.seg_id1;
            wr16(k, inf + 2, k.seg_id1);
        }
    }
    uint64_t cs = ~(uint64_t)rd16(k, k.udp + 6) + udp_res + 1;
    wr16(k, k.udp + 6, fold_checksum(cs));
}

// The rewrite's only stores into the SCION path after PathMeta are the SegIDs at INF+2 and, on a
// segment switch, INF+10.  With CurrINF past the info fields (parse_scion_path does not bound
// it) either can fall inside the hop field whose MAC is checked; the BPF code read that
// macinput before the rewrite (path_processing.h:39-57), so the bytes it would have seen are
// kept here and substituted at the check (mac_b8).
__device__ __forceinline__ void keep_mac_bytes(BrFrame &k)
{
    const int a = k.inf + 2, b = k.inf + 10, lo = k.mac_hf + 1, hi = k.mac_hf + 11;   // hop-field bytes read
    const bool wb = k.segment_switch && k.inf + 16 <= k.len;
    k.clob = (a + 1 >= lo && a <= hi ? 1u : 0u) | (wb && b + 1 >= lo && b <= hi ? 2u : 0u);
    if (k.clob) k.orig_ab = rd16(k, a) | ((k.clob & 2u) ? rd16(k, b) << 16 : 0u);
}

__device__ __forceinline__ uint32_t mac_b8(const BrFrame &k, int off)
{
    if ((k.clob & 1u) && (off == k.inf + 2 || off == k.inf + 3)) return (k.orig_ab >> (8 * (off - k.inf - 2))) & 0xffu;
    if ((k.clob & 2u) && (off == k.inf + 10 || off == k.inf + 11))
        return (k.orig_ab >> (16 + 8 * (off - k.inf - 10))) & 0xffu;
    return rd8(k, off);
}
__device__ __forceinline__ uint32_t mac_b16(const BrFrame &k, int off) { return mac_b8(k, off) | (mac_b8(k, off + 1) << 8); }

// ---- xdp.c: process_packet -----------------------------------------------------------------
// Returns the action (> 0 ends the frame), 0 (fall through to the MAC check without a record:
// the bare `return 0`/ABORT paths) or -1 (rewritten, go to the MAC check).
template <bool STATS>
__device__ __forceinline__ int process_packet(BrFrame &k)
{
    k.egress_ifindex = -1;
    int off = parse_underlay(k);
    if (off < 0) return (int)record<STATS>(k, k.verdict);
    off = parse_scion(k, off);
    if (off < 0) return (int)record<STATS>(k, k.verdict);

    uint32_t as_ing_ifid = 0;
    if (int_iface(k.ifindex) < 0) {
        int e = ingress_lookup(k);
        if (e < 0) return (int)record<STATS>(k, V_NO_INTERFACE);
        as_ing_ifid = s_br.ingress[e].ifid;
        uint32_t hf_ing = cons_at(k, k.inf) ? rd16(k, k.hf + 2) : rd16(k, k.hf + 4);
        if (sw16(hf_ing) != as_ing_ifid) return (int)record<STATS>(k, V_NO_INTERFACE);
    }
    if (as_ing_ifid != 0)   // path_type == SCION after parse_scion
        if (!as_ingress(k)) return (int)record<STATS>(k, k.verdict);

    int inf = k.inf;
    if (k.segment_switch) {
        inf += 8;
        if (beyond(k, inf + 8)) return 0;
    }
    uint32_t key = sw16(cons_at(k, inf) ? rd16(k, k.hf + 4) : rd16(k, k.hf + 2));
    int f = egress_lookup(key);
    if (f < 0) return (int)record<STATS>(k, V_ABORT);
    const DevBrEgress &fwd = s_br.egress[f];

    // The three next-hop cases (fib_lookup_as_egress / fib_lookup_egress_br / fib_lookup_ip,
    // fib.h) share one route-result step and one address update, so a wave holding frames of
    // several cases runs those once.
    const bool ext = fwd.fwd_external, sib = !ext && as_ing_ifid != 0;
    if (ext && !as_egress(k, as_ing_ifid)) return (int)record<STATS>(k, k.verdict);
    int r;
    if (ext || sib) {
        if (fwd.family != k.family) return (int)record<STATS>(k, V_UNDERLAY_MISMATCH);
        r = fwd.route;   // route_lookup of the link's remote address, resolved with the tables
    } else {
        r = ip_route(k);
    }
    if (!fib_result(k, r)) return (int)record<STATS>(k, k.verdict);
    const int egress = r >= 0 ? (int)s_br.routes[r].ifindex : 0;
    if (sib) {   // the sibling's packets leave from the internal interface on the route
        const int s = fwd.sib_iface;   // int_iface(egress)
        if (s < 0) return (int)record<STATS>(k, V_ABORT);
        if (s_br.int_ifaces[s].family != k.family) return (int)record<STATS>(k, V_UNDERLAY_MISMATCH);
    }
    k.nh = ext ? 1u : sib ? 2u : 0u;
    k.fwd = f;
    k.sib_if = fwd.sib_iface;
    if (k.need_mac) keep_mac_bytes(k);
    rewrite(k);
    k.egress_ifindex = egress;
    return -1;
}

__device__ __forceinline__ bool tx_port(int ifindex)
{
    if (ifindex < 0 || ifindex >= HFV_BR_MAX_TXPORTS) return false;
    return (s_br.tx_bits[ifindex >> 5] >> (ifindex & 31)) & 1u;
}

// ---- kernel ------------------------------------------------------------------------------------
template <bool STATS>
__device__ __forceinline__ void br_frame(BrFrame &k, uint64_t i, const DevKeyTable *keys,
                                         uint8_t *__restrict__ action, uint8_t *__restrict__ verdict,
                                         int32_t *__restrict__ egress, BrProf &prof)
{
    int a = process_packet<STATS>(k);
    prof.mark(1);
    if (k.cut) {   // headers reach past the window: untouched, uncounted, caller re-runs it whole
        action[i] = HFV_BR_ACTION_RETRY;
        verdict[i] = 0;
        egress[i] = -1;
        return;
    }
    if (a <= 0) {
        // border_router, xdp.c:256-283: the deferred MAC check, then the redirect
        uint32_t v = A_ABORTED;
        bool ok = true;
        if (k.need_mac && !s_br.hf_check_off) {
            // slot-0 key (xdp.c:82) through the scalar cache, only where a hop field is checked
            const int inf = k.mac_inf, hf = k.mac_hf;
            uint32_t mi[4], mac_lo, mac_hi;
            mi[0] = (k.mac_beta & 0xffffu) << 16;
            mi[1] = rd32(k, inf + 4);
            if (!k.clob) {
                mi[2] = (rd8(k, hf + 1) << 8) | (rd16(k, hf + 2) << 16);
                mi[3] = rd16(k, hf + 4);
                mac_lo = rd32(k, hf + 6);
                mac_hi = rd16(k, hf + 10);
            } else {   // the hop field overlaps the rewritten SegIDs: the bytes from before the rewrite
                mi[2] = (mac_b8(k, hf + 1) << 8) | (mac_b16(k, hf + 2) << 16);
                mi[3] = mac_b16(k, hf + 4);
                mac_lo = mac_b16(k, hf + 6) | (mac_b16(k, hf + 8) << 16);
                mac_hi = mac_b16(k, hf + 10);
            }
            const UniformKey ukey(keys);
            uint32_t t0, t1;
            const Lane l = lane_bases3();   // formed here: none of it stays live through the parse
            cmac48_macinput<3>(mi, ukey, l, t0, t1);
            ok = ukey.ok && t0 == mac_lo && (t1 & 0xffffu) == mac_hi;
        }
        if (!ok) v = V_INVALID_HF;
        else if (tx_port(k.egress_ifindex)) v = V_FORWARD;
        a = (int)record<STATS>(k, v);
    }
    action[i] = (uint8_t)a;
    verdict[i] = (uint8_t)k.last_verdict;
    egress[i] = k.egress_ifindex;
}

// One wave = one tile of 64 consecutive frames (lane = frame).  WIN > 0: the tile's first WIN
// header bytes per frame are fetched with coalesced 16-byte loads (WIN / 16 frames' chunks per
// wave instruction... 64 / (WIN / 16) frames per instruction), staged in LDS and parsed from
// there, and the next tile's bytes are already in flight while this one is parsed.
template <int BLOCK, bool STATS, int WIN>
__global__ __launch_bounds__(BLOCK) void k_br_process(const DevState *__restrict__ st, const uint8_t *pkts,
                                                      uint8_t *out,
                                                      uint64_t slot, uint32_t maxlen, uint32_t window,
                                                      const uint16_t *__restrict__ lens,
                                                      const uint32_t *__restrict__ ifidx, uint64_t n,
                                                      uint8_t *__restrict__ action, uint8_t *__restrict__ verdict,
                                                      int32_t *__restrict__ egress,
                                                      unsigned long long *__restrict__ stats)
{
    static_assert(WIN == 0 || (WIN == kBrWin && BLOCK / 64 <= kBrStageWaves), "staging geometry");
    constexpr int C = WIN > 0 ? WIN / 16 : 1;   // 16-byte chunks per frame
    fill_ttab<3>();   // 32 KiB (AES is a small part of the router's work; LDS goes to header rows)
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(&st->br);
        uint4 *dst = reinterpret_cast<uint4 *>(&s_br);
        for (uint32_t e = threadIdx.x; e < sizeof(DevBrConfig) / 16; e += BLOCK) dst[e] = src[e];
    }
    if constexpr (STATS)
        for (uint32_t e = threadIdx.x; e < HFV_BR_STATS_IFINDEX * 2 * HFV_BR_COUNTERS; e += BLOCK) s_stats[e] = 0;
    if (threadIdx.x == 0) s_br_next = 0;
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
    const uint64_t ntiles = (n + 63) / 64, nwaves = (uint64_t)gridDim.x * (BLOCK / 64);
    // Tiles go round the blocks first (wave w of block b starts at tile w * grid + b), so a
    // launch of fewer tiles than waves (the config-5 loop's 64 Ki-frame chunks: 1024 tiles)
    // still spreads over every CU instead of filling a quarter of them with 16 waves each.
    // (wave-uniform as far as the compiler knows: the buffer resources built from it stay in SGPRs)
    uint64_t t = (uint64_t)__builtin_amdgcn_readfirstlane(wib) * gridDim.x + blockIdx.x;
    if (s_br.detached) {   // `hfv-loader detach`: no router on the interface, every frame goes up the stack
        for (; t < ntiles; t += nwaves) {
            const uint64_t i = t * 64 + lane;
            if (i < n) {
                action[i] = A_PASS;
                verdict[i] = 0;
                egress[i] = -1;
            }
        }
        return;   // block-uniform: no barrier below is reached by only part of the block
    }
    const uint32_t fr_of = lane / C, ch = lane % C;   // staging: frame within round, chunk
    // The tile's header rows and the lane's own length / ingress ifindex are loaded at the top
    // of each tile, with no register prefetch of the next tile: the other waves of the CU (16
    // in the staged launch) hide the latency, and the prefetch's extra registers pushed the
    // 12-wave kernel into scratch spills (measured 152 us against 121 us); pulling
    // the next tile into L2 with one dword load per frame was 8 % slower (its load sits in the
    // in-order vmcnt queue of the current tile, profiles/r02/br_ab/pf_lane_w16_ab_r02c1.log).
    uint4 pre[C];
    uint32_t pre_len = 0, pre_ifx = 0;
    auto fetch = [&](uint64_t tt) {
        if constexpr (WIN > 0) {
#pragma unroll
            for (int r = 0; r < C; ++r) {
                uint64_t fi = tt * 64 + (uint64_t)(r * (64 / C)) + fr_of;
                if (fi >= n) fi = n - 1;   // unconditional (counted vmcnt); masked at use
                pre[r] = *reinterpret_cast<const uint4 *>(pkts + fi * slot + 16 * ch);
            }
        }
        uint64_t fi = tt * 64 + lane;
        if (fi >= n) fi = n - 1;
        pre_len = lens[fi];
        pre_ifx = ifidx[fi];
    };
    // HFV_BR_WB == 1: the same loads as buffer loads from a wave-uniform tile base (one lane
    // offset for all C chunks; lanes past the batch read zeros instead of a clamped frame)
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    typedef uint32_t v2u __attribute__((ext_vector_type(2)));
    const uint32_t voff = fr_of * (uint32_t)slot + 16u * ch;
    auto fetch_buf = [&](uint64_t tt) {
        // past the last tile: a zero-sized range (every load returns zeros, no memory access), so
        // the loop can issue the next tile's loads unconditionally
        const uint64_t left = tt * 64 < n ? n - tt * 64 : 0;
        const uint32_t nf = left < 64 ? (uint32_t)left : 64u;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(pkts) + tt * 64 * slot, 0, (int)(nf * (uint32_t)slot), 0x00020000);
#pragma unroll
        for (int r = 0; r < C; ++r) {
            // the whole offset in the VGPR: the bounds check does not cover soffset
            const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(voff + r * (64 / C) * (uint32_t)slot), 0, 0);
            pre[r] = make_uint4(v.x, v.y, v.z, v.w);
        }
        uint64_t fi = tt * 64 + lane;
        if (fi >= n) fi = n - 1;
        pre_len = lens[fi];
        pre_ifx = ifidx[fi];
    };
    BrProf prof;
    constexpr bool kEarly = WIN > 0 && HFV_BR_WB == 1;
    constexpr bool kDyn = kEarly && HFV_BR_DYN;
    // kDyn: this block's tiles [tb0, tb1), handed out by s_br_next (ntiles: nothing left)
    const uint64_t tb0 = ntiles * blockIdx.x / gridDim.x, tb1 = ntiles * (blockIdx.x + 1) / gridDim.x;
    auto claim = [&]() -> uint64_t {
        uint32_t g = 0;
        if (lane == 0) g = __hip_atomic_fetch_add(&s_br_next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint64_t tt = tb0 + __builtin_amdgcn_readfirstlane(g);
        return tt < tb1 ? tt : ntiles;
    };
    if constexpr (kDyn) t = claim();
    uint64_t tnext = t + nwaves;
    if constexpr (kEarly) {
        if (t < ntiles) fetch_buf(t);
        // (a builtin, so the waitcnt pass knows: the loop's vmcnt(C) assumes C younger stores)
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0) expcnt(7) lgkmcnt(15)
    }
    for (; t < ntiles; t = kDyn ? tnext : t + nwaves) {
        prof.start();
        if constexpr (!kEarly) fetch(t);
        if constexpr (kEarly) {
            // the loads of this tile were issued at the end of the previous one, before its C
            // write-back stores: wait for everything but those stores
            __builtin_amdgcn_s_waitcnt(0x0F70 | C);   // vmcnt(C) expcnt(7) lgkmcnt(15)
        }
        if constexpr (WIN > 0) {
            uint32_t *rows = s_hdr + wib * 64 * kBrRow;
#pragma unroll
            for (int r = 0; r < C; ++r) {
                uint32_t *d = rows + (r * (64 / C) + fr_of) * kBrRow + 4 * ch;
                d[0] = pre[r].x; d[1] = pre[r].y; d[2] = pre[r].z; d[3] = pre[r].w;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        const uint32_t len = pre_len, ifx = pre_ifx;
        if constexpr (HFV_BR_PROF) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        prof.mark(0);
        uint64_t i = t * 64 + lane;
        uint32_t dirty = 0;
        if (i < n) {
            BrFrame k = {};
            k.p = pkts + i * slot;
            k.po = out + i * slot;
            k.win = WIN;
            k.row = (wib * 64 + lane) * kBrRow;
            k.len = (int)(len <= maxlen ? len : maxlen);
            k.lim = k.len < (int)window ? k.len : (int)window;
            k.ifindex = ifx;
            if constexpr (kEarly && HFV_BR_EXT) {
                // the SCION header's end by its HdrLen (sc + 5; sc after Ethernet, IPv4 with its
                // IHL or IPv6, and UDP): a hint only, every read still checks its own bounds
                const uint32_t proto = lds_u16_at(k, 12);
                const int udp = proto == 0x0008u ? 14 + 4 * (int)(lds_u16_at(k, 14) & 0x0fu) : 54;
                const int sc = udp + 8;
                const int end = sc + 4 * (int)(reinterpret_cast<const uint8_t *>(s_hdr + k.row)[sc + 5 < WIN ? sc + 5 : 0]);
                k.has_ext = k.lim > WIN && sc + 5 < WIN && end > WIN && (proto == 0x0008u || proto == 0xdd86u);
                const uint64_t left = n - t * 64;
                const uint32_t nf = left < 64 ? (uint32_t)left : 64u;
                const __amdgpu_buffer_rsrc_t rx =
                    __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(pkts) + t * 64 * slot, 0, (int)(nf * (uint32_t)slot), 0x00020000);
                const v2u e = __builtin_amdgcn_raw_buffer_load_b64(rx, (int)(k.has_ext ? lane * (uint32_t)slot + WIN : 0x80000000u), 0, 0);
                k.ext[0] = e.x; k.ext[1] = e.y;
            }
            br_frame<STATS>(k, i, &st->keys, action, verdict, egress, prof);
            dirty = k.dirty;
        }
        prof.mark(2);
        if constexpr (WIN > 0) {
            // write the rewritten 16-byte chunks back (WIN / 16 lanes per frame, each storing its
            // chunk if the frame's lane wrote into it): untouched chunks stay clean in L2, so a
            // frame whose changes lie in one 32-byte sector of a line costs that sector, not the line
            uint32_t cmask[C];
#pragma unroll
            for (int r = 0; r < C; ++r) cmask[r] = (uint32_t)__shfl((int)dirty, r * (64 / C) + (int)fr_of);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t *rows = s_hdr + wib * 64 * kBrRow;
            if constexpr (HFV_BR_WB == 1) {
                // the next tile's loads go to registers (the rows are read below, then restaged at
                // the top of the next iteration), ahead of this tile's stores
                tnext = kDyn ? claim() : t + nwaves;
                fetch_buf(tnext);
                const __amdgpu_buffer_rsrc_t rs =
                    __builtin_amdgcn_make_buffer_rsrc(out + t * 64 * slot, 0, (int)(64u * (uint32_t)slot), 0x00020000);
#pragma unroll
                for (int r = 0; r < C; ++r) {
                    const uint32_t fr = r * (64 / C) + fr_of;
                    const uint32_t *q = rows + fr * kBrRow + 4 * ch;
                    const v4u q4 = v4u{q[0], q[1], q[2], q[3]};
                    const uint32_t off = ((cmask[r] >> ch) & 1u) ? voff + r * (64 / C) * (uint32_t)slot : 0x80000000u;
                    __builtin_amdgcn_raw_buffer_store_b128(q4, rs, (int)off, 0, 0);
                }
            } else if constexpr (HFV_BR_WB == 0) {
#pragma unroll
                for (int r = 0; r < C; ++r) {
                    uint32_t fr = r * (64 / C) + fr_of;
                    if ((cmask[r] >> ch) & 1u) {
                        const uint32_t *q = rows + fr * kBrRow + 4 * ch;
                        *reinterpret_cast<uint4 *>(out + (t * 64 + fr) * slot + 16 * ch) = make_uint4(q[0], q[1], q[2], q[3]);
                    }
                }
            }
        }
        if constexpr (WIN > 0) {   // every lane is done with the rows before they are restaged
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if constexpr (HFV_BR_PROF) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        prof.mark(3);
        prof.c[4] += 1;
    }
#if HFV_BR_PROF
    if (lane == 0)
        for (int q = 0; q < 5; ++q) atomicAdd(&g_br_prof[q], (unsigned long long)prof.c[q]);
#endif
    if constexpr (STATS) {
        __syncthreads();
        for (uint32_t e = threadIdx.x; e < HFV_BR_STATS_IFINDEX * 2 * HFV_BR_COUNTERS; e += BLOCK) {
            unsigned long long v = (unsigned long long)s_stats[e];
            if (v) atomicAdd(stats + e, v);
        }
    }
}

#if HFV_BR_PROF
// diagnostics: the phase counters of the kernels run since the last call (then cleared)
extern "C" int hfv_debug_br_prof(unsigned long long out[8])
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_br_prof), 8 * sizeof(unsigned long long)) != hipSuccess) return -1;
    static const unsigned long long zero[8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_br_prof), zero, sizeof zero) == hipSuccess ? 0 : -1;
}
#endif

int launch_br_process(const LaunchGeom &g, const DevState *st, uint8_t *pkts, size_t slot, uint32_t maxlen,
                      uint32_t window, const uint16_t *len, const uint32_t *ingress_ifindex, size_t n,
                      uint8_t *action, uint8_t *verdict, int32_t *egress_ifindex, uint64_t *stats, void *stream,
                      void *ev_start, void *ev_stop, uint8_t *out)
{
    // `out` (default: in place) receives only the bytes the router changes; the caller keeps the
    // rest of each frame there.  No byte is read after the router wrote it (the macinput bytes a
    // SegID store can overwrite are kept before it, keep_mac_bytes), so reading `pkts` while
    // writing `out` gives the in-place result.
    if (!out) out = pkts;
    // Staged variant when the 16-byte header loads are aligned and in bounds, the direct one
    // otherwise.  Persistent grid: one block per CU (LDS: tables + counters [+ header rows]).
    // (the staged loop addresses a tile of 64 slots through 32-bit buffer offsets: 64 * slot < 2^31)
    bool staged = slot >= (size_t)kBrWin && slot % 16 == 0 && ((uintptr_t)pkts & 15) == 0 &&
                  ((uintptr_t)out & 15) == 0 && slot < ((size_t)1 << 25);
    using K = void (*)(const DevState *, const uint8_t *, uint8_t *, uint64_t, uint32_t, uint32_t,
                       const uint16_t *,
                       const uint32_t *, uint64_t, uint8_t *, uint8_t *, int32_t *, unsigned long long *);
    K k;
    int block;
    if (staged) {
        block = kBrStageWaves * 64;
        k = stats ? k_br_process<kBrStageWaves * 64, true, kBrWin> : k_br_process<kBrStageWaves * 64, false, kBrWin>;
    } else {
        block = 1024;
        k = stats ? k_br_process<1024, true, 0> : k_br_process<1024, false, 0>;
    }
#if HFV_BR_STATS32
    // 32-bit block counters: split a launch whose blocks could count 2^32 bytes of one kind
    // (a block's frames x the largest length); every launch adds into the same counters
    if (stats) {
        const uint64_t per_block = (uint64_t)(UINT32_MAX / (maxlen ? maxlen : 1));   // frames
        // a block's range is ceil(tiles / grid) tiles at most, i.e. up to a tile more than the even
        // share plus a tile of rounding: reserve two tiles
        uint64_t cap_n = (per_block > 128 ? per_block - 128 : 1) * (uint64_t)g.num_cus;
        if (g.br_split_cap && g.br_split_cap < cap_n) cap_n = g.br_split_cap;   // test build only
        if ((uint64_t)n > cap_n) {
            for (size_t off = 0; off < n; off += cap_n) {
                const size_t m = n - off < cap_n ? n - off : (size_t)cap_n;
                int e = launch_br_process(g, st, pkts + off * slot, slot, maxlen, window, len + off, ingress_ifindex + off, m,
                                          action + off, verdict + off, egress_ifindex + off, stats, stream,
                                          off == 0 ? ev_start : nullptr, off + m >= n ? ev_stop : nullptr,
                                          out + off * slot);
                if (e) return e;
            }
            return 0;
        }
    }
#endif
    const uint64_t tiles = (n + 63) / 64, cap = (uint64_t)g.num_cus;   // one block per CU at most
    unsigned grid = (unsigned)(tiles < cap ? (tiles ? tiles : 1) : cap);
    if (g.br_grid_cap && g.br_grid_cap < grid) grid = g.br_grid_cap;   // test build only
    hipExtLaunchKernelGGL(k, dim3(grid), dim3(block), 0, (hipStream_t)stream, (hipEvent_t)ev_start,
                          (hipEvent_t)ev_stop, 0u, st, (const uint8_t *)pkts, out, (uint64_t)slot, maxlen,
                          window, len, ingress_ifindex, (uint64_t)n, action, verdict, egress_ifindex,
                          (unsigned long long *)stats);
    return (int)hipGetLastError();
}

}  // namespace hfv
