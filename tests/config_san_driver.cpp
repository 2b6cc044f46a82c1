// The router-configuration path for C callers (csrc/hfv_config.cpp: br-loader's TOML and
// topology.json parsers and the table builder, hfv_br_config_load; the pinned router-table
// file) built with AddressSanitizer + UBSan and driven over the reference's configurations and
// over mutated copies of them (truncations, byte flips, inserted and deleted characters,
// swapped lines): every call must return a status and a diagnostic, never crash, leak or read
// out of bounds (tests/test_sanitize.py).  Usage: config_san_driver <fixture dir> <tmp dir>.
#include <errno.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <string>
#include <vector>

#include "scion_hfv.h"

namespace hfv {
int fail(int code, const char *fmt, ...)   // the library's error sink lives in hfv_api.cpp
{
    va_list ap;
    va_start(ap, fmt);
    char buf[256];
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    return code;
}
}  // namespace hfv

#define CHECK(c)                                                                 \
    do {                                                                         \
        if (!(c)) {                                                              \
            fprintf(stderr, "%s:%d check failed: %s\n", __FILE__, __LINE__, #c); \
            abort();                                                             \
        }                                                                        \
    } while (0)

static std::string slurp(const std::string &p)
{
    FILE *f = fopen(p.c_str(), "rb");
    CHECK(f);
    std::string s;
    char buf[4096];
    size_t k;
    while ((k = fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, k);
    fclose(f);
    return s;
}

static void spit(const std::string &p, const std::string &s)
{
    FILE *f = fopen(p.c_str(), "wb");
    CHECK(f);
    CHECK(fwrite(s.data(), 1, s.size(), f) == s.size());
    fclose(f);
}

static hfv_br_ifaddr ifa(const char *name, uint32_t index, uint8_t a, uint8_t b, uint8_t c, uint8_t d)
{
    hfv_br_ifaddr x = {};
    snprintf(x.ifname, sizeof x.ifname, "%s", name);
    x.ifindex = index;
    x.family = HFV_AF_INET;
    x.addr[0] = a; x.addr[1] = b; x.addr[2] = c; x.addr[3] = d;
    return x;
}

static int load(const std::string &toml, const std::vector<hfv_br_ifaddr> &ifs, hfv_br_config *cfg, std::string *diag)
{
    static char self[256], listing[16384], dg[16384];
    const hfv_br_next_hop hop = {HFV_AF_INET, {10, 1, 1, 1}, 32, "veth1", {2, 0, 0, 0, 0, 1}, {2, 0, 0, 0, 0, 0}, 0};
    int rc = hfv_br_config_load(toml.c_str(), ifs.data(), ifs.size(), &hop, 1, cfg, self, sizeof self, listing,
                                sizeof listing, dg, sizeof dg);
    CHECK(strnlen(self, sizeof self) < sizeof self && strnlen(listing, sizeof listing) < sizeof listing &&
          strnlen(dg, sizeof dg) < sizeof dg);
    if (diag) *diag = dg;
    return rc;
}

static std::string mutate(std::string s, std::mt19937_64 &rng)
{
    const int kind = (int)(rng() % 6);
    if (s.empty()) return "x";
    const size_t at = rng() % s.size();
    switch (kind) {
    case 0: return s.substr(0, at);                                                    // truncate
    case 1: s[at] = (char)(rng() & 0xff); return s;                                     // flip a byte
    case 2: s.insert(at, 1, "[]{}\",=:#\n\\0.-e"[rng() % 16]); return s;                // insert syntax
    case 3: s.erase(at, 1 + rng() % 8); return s;                                       // delete a run
    case 4: {                                                                           // swap two lines
        std::vector<std::string> lines;
        size_t p = 0, q;
        while ((q = s.find('\n', p)) != std::string::npos) { lines.push_back(s.substr(p, q - p + 1)); p = q + 1; }
        lines.push_back(s.substr(p));
        std::swap(lines[rng() % lines.size()], lines[rng() % lines.size()]);
        std::string o;
        for (auto &l : lines) o += l;
        return o;
    }
    default: s.insert(at, std::string(1 + rng() % 300, (char)('0' + rng() % 10))); return s;   // long number
    }
}

int main(int argc, char **argv)
{
    CHECK(argc == 3);
    const std::string fix = argv[1], tmp = argv[2];
    const std::vector<hfv_br_ifaddr> ifs = {ifa("veth1", 1, 10, 1, 1, 2), ifa("veth3", 3, 10, 1, 2, 2),
                                            ifa("veth5", 5, 10, 2, 0, 1), ifa("veth7", 7, 10, 2, 0, 3)};
    hfv_br_config cfg;
    std::string diag;
    // the reference's configurations load (topology paths rewritten to the fixture copies)
    const std::string topo = slurp(fix + "/topology.json");
    const std::string topo_path = tmp + "/topology.json";
    spit(topo_path, topo);
    std::vector<std::string> tomls;
    for (const char *name : {"br1.toml", "br2.toml", "br3.toml"}) {
        std::string t = slurp(fix + "/" + name);
        const size_t p = t.find("br_config/topology.json");
        CHECK(p != std::string::npos);
        t.replace(p, strlen("br_config/topology.json"), topo_path);
        tomls.push_back(t);
        const std::string path = tmp + "/" + name;
        spit(path, t);
        CHECK(load(path, ifs, &cfg, &diag) == 0);
    }
    // mutated configurations and topologies: a status and a diagnostic, nothing else
    std::mt19937_64 rng(0x5C10C0F1);
    int ok = 0, rejected = 0;
    const std::string mt = tmp + "/m.toml", mj = tmp + "/m.json";
    for (int it = 0; it < 3000; ++it) {
        std::string t = tomls[it % tomls.size()], j = topo;
        if (it % 2 == 0) {
            t = mutate(t, rng);
            if (rng() % 4 == 0) t = mutate(t, rng);
        } else {
            j = mutate(j, rng);
            if (rng() % 4 == 0) j = mutate(j, rng);
        }
        const size_t p = t.find(topo_path);
        if (p != std::string::npos) t.replace(p, topo_path.size(), mj);
        spit(mt, t);
        spit(mj, j);
        const int rc = load(mt, ifs, &cfg, &diag);
        CHECK(rc == 0 || rc < 0);
        if (rc == 0) ++ok;
        else {
            ++rejected;
            CHECK(!diag.empty());
        }
    }
    CHECK(ok > 0 && rejected > 0);
    // pinned router tables: publish, read back, republish
    const std::string pin = tmp + "/br_config";
    CHECK(load(tmp + "/br1.toml", ifs, &cfg, &diag) == 0);
    CHECK(hfv_brconfig_publish(pin.c_str(), &cfg) == 0);
    hfv_br_config back;
    CHECK(hfv_brconfig_read(pin.c_str(), &back) == 0);
    CHECK(memcmp(&cfg, &back, sizeof cfg) == 0);
    CHECK(load(tmp + "/br2.toml", ifs, &cfg, &diag) == 0);
    CHECK(hfv_brconfig_publish(pin.c_str(), &cfg) == 0);
    CHECK(hfv_brconfig_read(pin.c_str(), &back) == 0);
    CHECK(memcmp(&cfg, &back, sizeof cfg) == 0);
    CHECK(hfv_brconfig_read((tmp + "/missing").c_str(), &back) < 0);
    printf("config san ok: %d loaded, %d rejected\n", ok, rejected);
    return 0;
}
