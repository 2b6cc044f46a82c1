// hfv-loader -- control-plane CLI for the MI355X hop-field verifier, the counterpart of the
// reference's `br-loader key add|remove` (br/src/br_loader.cpp:50-61, 182-295).
//
//   hfv-loader key add <br> <index> <base64-key>    decode, expand, derive K1, update map (any u32
//                                                   index, at most 8 keys: the reference map's
//                                                   semantics, maps.h:60-67; 0..255 and 256 keys
//                                                   in a map `attach --key-slots` created)
//   hfv-loader key remove <br> <index>              erase the slot (it then fails closed)
//   hfv-loader key list <br>                        print occupied slots and K1 of each
//   hfv-loader watch <br> <iface> [seconds]         verdict counters of one ingress port,
//                                                   every second (br_loader.cpp:162-180)
//   hfv-loader attach <config> [--route R]...       loadConfig + initializeMaps + pin
//                                                   (attachBr, br_loader.cpp:88-151): print the
//                                                   configuration, publish the router tables to
//                                                   $HFV_PIN_DIR/<self>/br_config, create (or
//                                                   reuse) the pinned key and counter maps.
//                                                   R = <prefix>/<len>,<iface>,<smac>,<dmac>[,<ret>]
//                                                   is one static next hop (bpf_fib_lookup has no
//                                                   GPU counterpart)
//   hfv-loader detach <br>                          unpublish the router tables (detachBr)
//
// The pinned map lives at $HFV_PIN_DIR/<br>/mac_key_map (default /dev/shm/hfv); a data plane
// that called hfv_ctx_attach_keymap() on it picks the change up at its next batch.  Messages
// and exit codes follow br-loader: errors on stderr, EXIT_FAILURE.
#include <arpa/inet.h>
#include <net/if.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <stdexcept>
#include <string>

#include "../../include/scion_hfv.h"

static void print_usage()
{
    fprintf(stderr,
            "Usage: hfv-loader key add <br> <index> <key>\n"
            "                  key remove <br> <index>\n"
            "                  key list <br>\n"
            "       hfv-loader watch <br> <iface> [seconds]\n"
            "       hfv-loader attach <config> [--key-slots] [--no-ipv4] [--no-ipv6] [--no-scion-path]\n"
            "                         [--route <prefix>/<len>,<iface>,<smac>,<dmac>[,<ret>]]...\n"
            "                  detach <br>\n");
}

static bool parse_index(const char *s, uint32_t *out)
{
    try {
        size_t pos = 0;
        unsigned long v = std::stoul(std::string(s), &pos);
        if (pos != strlen(s) || v > 0xffffffffUL) return false;
        *out = (uint32_t)v;
        return true;
    } catch (const std::exception &) {
        return false;
    }
}

static int map_path(const char *br, char *path, size_t len)
{
    if (hfv_keymap_path(br, path, len) != 0) {
        fprintf(stderr, "Invalid border router name: %s\n", hfv_last_error());
        return -1;
    }
    return 0;
}

static int add_key(int argc, char **argv)
{
    if (argc < 3) { print_usage(); return EXIT_FAILURE; }
    char path[4096];
    if (map_path(argv[0], path, sizeof path)) return EXIT_FAILURE;
    uint32_t index;
    if (!parse_index(argv[1], &index)) {
        fprintf(stderr, "Invalid verification key index\n");
        return EXIT_FAILURE;
    }
    struct aes_key key;
    if (hfv_decode_key_b64(argv[2], &key) != 0) {
        fprintf(stderr, "Invalid MAC verification key: %s\n", hfv_last_error());
        return EXIT_FAILURE;
    }
    // the same derivation as br_loader.cpp:213-218: expansion, subkeys, keep K1
    struct hop_key hk;
    aes_key_expansion(&key, &hk.key);
    struct aes_block subkeys[2];
    aes_cmac_subkeys(&hk.key, subkeys);
    hk.subkey = subkeys[0];
    // a map this command has to create gets the reference map's semantics (u32 index, at most
    // 8 entries, maps.h:60-67); one `attach --key-slots` created keeps its 256 direct slots
    if (hfv_keymap_create_mode(path, HFV_KEYMAP_HASH8) != 0 || hfv_keymap_update(path, index, &hk) != 0) {
        fprintf(stderr, "Update failed: %s\n", hfv_last_error());
        return EXIT_FAILURE;
    }
    return EXIT_SUCCESS;
}

static int remove_key(int argc, char **argv)
{
    if (argc < 2) { print_usage(); return EXIT_FAILURE; }
    char path[4096];
    if (map_path(argv[0], path, sizeof path)) return EXIT_FAILURE;
    uint32_t index;
    if (!parse_index(argv[1], &index)) {
        fprintf(stderr, "Invalid verification key index\n");
        return EXIT_FAILURE;
    }
    if (hfv_keymap_erase(path, index) != 0) {
        fprintf(stderr, "Update failed: %s\n", hfv_last_error());
        return EXIT_FAILURE;
    }
    return EXIT_SUCCESS;
}

static int list_keys(int argc, char **argv)
{
    if (argc < 1) { print_usage(); return EXIT_FAILURE; }
    char path[4096];
    if (map_path(argv[0], path, sizeof path)) return EXIT_FAILURE;
    static uint32_t idx[HFV_MAX_KEYS + 8];
    static struct hop_key keys[HFV_MAX_KEYS + 8];
    size_t n = 0;
    if (hfv_keymap_list(path, idx, keys, HFV_MAX_KEYS + 8, &n) != 0) {
        fprintf(stderr, "Cannot read key map: %s\n", hfv_last_error());
        return EXIT_FAILURE;
    }
    for (size_t k = 0; k < n && k < HFV_MAX_KEYS + 8; ++k) {
        printf("%u K1=", idx[k]);
        for (int i = 0; i < 16; ++i) printf("%02x", keys[k].subkey.b[i]);
        printf("\n");
    }
    return EXIT_SUCCESS;
}

// ---- watch (stats.cpp:38-144) ------------------------------------------------------------
static const char *kStatNames[HFV_BR_COUNTERS] = {
    "Undefined",       "Forwarded",     "Parse error",       "Not SCION",    "Not implemented", "No interface",
    "Underlay mismatch", "Router alert", "FIB lookup drop", "FIB lookup pass", "Invalid HF",
};

static volatile sig_atomic_t g_stop = 0;
static void on_sigint(int) { g_stop = 1; }

static void print_stats(const uint64_t *bytes, const uint64_t *pkts, const double *rb, const double *rp)
{
    printf("Verdict             Packets    pkts/s         Bytes    Mbit/s\n");
    for (int i = 0; i < HFV_BR_COUNTERS; ++i)
        printf("%-18s%8llu%11.0f%14llu%10.5g\n", kStatNames[i], (unsigned long long)pkts[i], rp[i],
               (unsigned long long)bytes[i], rb[i] * 8e-6);
    fflush(stdout);
}

static bool port_totals(const char *path, uint32_t ifindex, uint64_t *bytes, uint64_t *pkts)
{
    static uint64_t all[HFV_BR_STATS_IFINDEX * 2 * HFV_BR_COUNTERS];
    if (hfv_statsmap_read(path, all) != 0) return false;
    memcpy(bytes, all + (size_t)ifindex * 2 * HFV_BR_COUNTERS, sizeof(uint64_t) * HFV_BR_COUNTERS);
    memcpy(pkts, all + ((size_t)ifindex * 2 + 1) * HFV_BR_COUNTERS, sizeof(uint64_t) * HFV_BR_COUNTERS);
    return true;
}

static double now_s()
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static int watch(int argc, char **argv)
{
    if (argc < 2) { print_usage(); return EXIT_FAILURE; }
    char path[4096];
    if (hfv_statsmap_path(argv[0], path, sizeof path) != 0) {
        fprintf(stderr, "Invalid border router name: %s\n", hfv_last_error());
        return EXIT_FAILURE;
    }
    uint32_t ifindex = if_nametoindex(argv[1]);
    if (!ifindex && !parse_index(argv[1], &ifindex)) {
        fprintf(stderr, "Unknown interface: %s\n", argv[1]);
        return EXIT_FAILURE;
    }
    if (ifindex >= HFV_BR_STATS_IFINDEX) {
        fprintf(stderr, "Lookup failed\n");
        return EXIT_FAILURE;
    }
    uint32_t seconds = 0;   // 0: until SIGINT, like br-loader
    if (argc >= 3 && !parse_index(argv[2], &seconds)) { print_usage(); return EXIT_FAILURE; }
    uint64_t b[HFV_BR_COUNTERS], p[HFV_BR_COUNTERS], pb[HFV_BR_COUNTERS], pp[HFV_BR_COUNTERS];
    double rb[HFV_BR_COUNTERS] = {0}, rp[HFV_BR_COUNTERS] = {0};
    double t0 = now_s();
    if (!port_totals(path, ifindex, b, p)) {
        fprintf(stderr, "Lookup failed\n");
        return EXIT_FAILURE;
    }
    print_stats(b, p, rb, rp);
    signal(SIGINT, on_sigint);
    for (uint32_t k = 0; !g_stop && (seconds == 0 || k < seconds); ++k) {
        sleep(1);
        if (g_stop) break;
        double t1 = now_s(), dt = t1 - t0;
        t0 = t1;
        memcpy(pb, b, sizeof b);
        memcpy(pp, p, sizeof p);
        if (!port_totals(path, ifindex, b, p)) {
            fprintf(stderr, "Lookup failed\n");
            break;
        }
        for (int i = 0; i < HFV_BR_COUNTERS; ++i) {
            rb[i] = (double)(b[i] - pb[i]) / dt;
            rp[i] = (double)(p[i] - pp[i]) / dt;
        }
        print_stats(b, p, rb, rp);
    }
    return EXIT_SUCCESS;
}

// ---- attach / detach (br_loader.cpp:88-160) ---------------------------------------------
static bool parse_mac(const char *s, uint8_t out[6])
{
    unsigned v[6];
    if (sscanf(s, "%x:%x:%x:%x:%x:%x", &v[0], &v[1], &v[2], &v[3], &v[4], &v[5]) != 6) return false;
    for (int i = 0; i < 6; ++i) {
        if (v[i] > 255) return false;
        out[i] = (uint8_t)v[i];
    }
    return true;
}

// <prefix>/<len>,<iface>,<smac>,<dmac>[,<ret>]
static bool parse_route(const char *arg, struct hfv_br_next_hop *h)
{
    memset(h, 0, sizeof *h);
    std::string a(arg);
    std::string f[5];
    int n = 0;
    size_t pos = 0;
    while (n < 5) {
        size_t c = a.find(',', pos);
        f[n++] = a.substr(pos, c == std::string::npos ? std::string::npos : c - pos);
        if (c == std::string::npos) break;
        pos = c + 1;
    }
    if (n < 4) return false;
    size_t slash = f[0].find('/');
    if (slash == std::string::npos) return false;
    std::string ip = f[0].substr(0, slash);
    uint32_t plen;
    if (!parse_index(f[0].c_str() + slash + 1, &plen)) return false;
    if (inet_pton(AF_INET, ip.c_str(), h->prefix) == 1) h->family = HFV_AF_INET;
    else if (inet_pton(AF_INET6, ip.c_str(), h->prefix) == 1) h->family = HFV_AF_INET6;
    else return false;
    if (plen > (h->family == HFV_AF_INET ? 32u : 128u) || f[1].empty() || f[1].size() >= sizeof h->ifname) return false;
    h->prefix_len = plen;
    memcpy(h->ifname, f[1].c_str(), f[1].size());
    if (!parse_mac(f[2].c_str(), h->smac) || !parse_mac(f[3].c_str(), h->dmac)) return false;
    if (n == 5) h->ret = atoi(f[4].c_str());
    return true;
}

static int attach(int argc, char **argv)
{
    if (argc < 1) { print_usage(); return EXIT_FAILURE; }
    static struct hfv_br_next_hop hops[HFV_BR_MAX_ROUTES];
    size_t nh = 0;
    int kmode = HFV_KEYMAP_HASH8;   // the reference's mac_key_map (maps.h:60-67)
    uint32_t disabled = 0;
    for (int i = 1; i < argc; ++i) {
        if (strcmp(argv[i], "--route") == 0 && i + 1 < argc && nh < HFV_BR_MAX_ROUTES && parse_route(argv[i + 1], &hops[nh])) {
            ++nh;
            ++i;
            continue;
        }
        if (strcmp(argv[i], "--key-slots") == 0) {   // 256 direct slots (per-interface keys)
            kmode = HFV_KEYMAP_SLOTS;
            continue;
        }
        // the reference's build options switched off (br/CMakeLists.txt:5-7)
        if (strcmp(argv[i], "--no-ipv4") == 0) { disabled |= HFV_BR_NO_IPV4; continue; }
        if (strcmp(argv[i], "--no-ipv6") == 0) { disabled |= HFV_BR_NO_IPV6; continue; }
        if (strcmp(argv[i], "--no-scion-path") == 0) { disabled |= HFV_BR_NO_SCION_PATH; continue; }
        fprintf(stderr, "Invalid argument: %s\n", argv[i]);
        print_usage();
        return EXIT_FAILURE;
    }
    static struct hfv_br_config cfg;
    static char self[256], listing[65536], diag[65536];
    int rc = hfv_br_config_load(argv[0], nullptr, 0, hops, nh, &cfg, self, sizeof self, listing, sizeof listing,
                                diag, sizeof diag);
    fputs(diag, stderr);
    if (rc) return EXIT_FAILURE;
    fputs(listing, stdout);
    fflush(stdout);
    // initializeMaps stores every address through STORE_IPV4/6, which throw for a family the
    // router is built without (maps.cpp:68-80); main prints "ERROR: ..." (br_loader.cpp:291-294)
    if (hfv_br_config_check_options(&cfg, disabled) != 0) {
        fprintf(stderr, "ERROR: %s\n", hfv_last_error());
        return EXIT_FAILURE;
    }
    char kpath[4096], spath[4096], cpath[4096];
    if (hfv_keymap_path(self, kpath, sizeof kpath) || hfv_statsmap_path(self, spath, sizeof spath) ||
        hfv_brconfig_path(self, cpath, sizeof cpath)) {
        fprintf(stderr, "Invalid border router name: %s\n", hfv_last_error());
        return EXIT_FAILURE;
    }
    // reusePinnedMap: keys and counters survive a re-attach (br_loader.cpp:119-126)
    if (access(kpath, F_OK) == 0) printf("Reusing pinned map: \"%s\"\n", kpath);
    else if (hfv_keymap_create_mode(kpath, kmode) != 0) {
        fprintf(stderr, "Cannot create key map: %s\n", hfv_last_error());
        return EXIT_FAILURE;
    }
    if (access(spath, F_OK) == 0) printf("Reusing pinned map: \"%s\"\n", spath);
    else {
        static uint64_t zero[HFV_BR_STATS_IFINDEX * 2 * HFV_BR_COUNTERS];
        if (hfv_statsmap_add(spath, zero) != 0) {
            fprintf(stderr, "Cannot create counter map: %s\n", hfv_last_error());
            return EXIT_FAILURE;
        }
    }
    if (hfv_brconfig_publish_opts(cpath, &cfg, disabled) != 0) {
        fprintf(stderr, "Cannot publish router tables: %s\n", hfv_last_error());
        return EXIT_FAILURE;
    }
    printf("HFV-BR attached: %s\n", cpath);
    return EXIT_SUCCESS;
}

static int detach(int argc, char **argv)
{
    if (argc < 1) { print_usage(); return EXIT_FAILURE; }
    char cpath[4096];
    if (hfv_brconfig_path(argv[0], cpath, sizeof cpath) != 0) {
        fprintf(stderr, "Invalid border router name: %s\n", hfv_last_error());
        return EXIT_FAILURE;
    }
    if (hfv_brconfig_detach(cpath) != 0) {   // the file stays: attached data planes see the flag
        fprintf(stderr, "Not attached: %s\n", cpath);
        return EXIT_FAILURE;
    }
    printf("HFV-BR detached\n");
    return EXIT_SUCCESS;
}

int main(int argc, char **argv)
{
    if (argc >= 2 && strcmp(argv[1], "attach") == 0) return attach(argc - 2, argv + 2);
    if (argc >= 2 && strcmp(argv[1], "detach") == 0) return detach(argc - 2, argv + 2);
    if (argc >= 2 && strcmp(argv[1], "watch") == 0) return watch(argc - 2, argv + 2);
    if (argc >= 3 && strcmp(argv[1], "key") == 0) {
        if (strcmp(argv[2], "add") == 0) return add_key(argc - 3, argv + 3);
        if (strcmp(argv[2], "remove") == 0) return remove_key(argc - 3, argv + 3);
        if (strcmp(argv[2], "list") == 0) return list_keys(argc - 3, argv + 3);
    }
    print_usage();
    return EXIT_FAILURE;
}
