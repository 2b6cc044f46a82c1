// hfv_config.cpp -- br-loader's configuration path for C callers: the router's TOML file and
// the SCION topology.json it names -> the router tables of hfv_br_process (struct
// hfv_br_config), and the pinned copy of those tables that `hfv-loader attach` publishes.
//
// Follows, with the same inputs, checks and messages:
//   loadConfig / parseTopology / parseInternalIfaces / parseUdpEp / getIfAddr
//                                                       br/src/config.cpp:50-262
//   operator<< (the "XDP Border Router ..." listing)    br/src/config.cpp:296-330
//   populateIngressMap / populateEgressMap / populateIntIfMap / populatePortMap
//                                                       br/src/maps.cpp:91-200
// toml++ and Boost.JSON (the reference's parsers) are not available here: the TOML subset a
// br-loader configuration uses (key = value, strings, integers, booleans, arrays, inline
// tables, [table] and [[array of tables]] headers, comments) and JSON are parsed by the small
// recursive-descent readers below.  bpf_fib_lookup has no GPU counterpart: next hops come
// as an explicit table (struct hfv_br_next_hop).
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <ifaddrs.h>
#include <net/if.h>
#include <netinet/in.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/file.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "hfv_internal.h"

namespace hfv {
namespace {

// ---- a parsed TOML or JSON value -------------------------------------------------------
struct Node {
    enum Kind { Null, Str, Int, Float, Bool, Arr, Obj } kind = Null;
    std::string s;
    long long i = 0;
    double d = 0;
    bool b = false;
    std::vector<Node> arr;
    std::vector<std::pair<std::string, Node>> obj;   // insertion order, as toml++ / Boost.JSON iterate
    const Node *get(const std::string &k) const
    {
        if (kind != Obj) return nullptr;
        for (const auto &kv : obj)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
    Node *get_mut(const std::string &k)
    {
        for (auto &kv : obj)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
};

struct ParseError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

static std::string fmt(const char *f, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, f);
    vsnprintf(buf, sizeof buf, f, ap);
    va_end(ap);
    return buf;
}

// UTF-8 encoding of a \u escape
static void put_utf8(std::string &o, unsigned cp)
{
    if (cp < 0x80) o += (char)cp;
    else if (cp < 0x800) { o += (char)(0xc0 | cp >> 6); o += (char)(0x80 | (cp & 0x3f)); }
    else if (cp < 0x10000) { o += (char)(0xe0 | cp >> 12); o += (char)(0x80 | ((cp >> 6) & 0x3f)); o += (char)(0x80 | (cp & 0x3f)); }
    else { o += (char)(0xf0 | cp >> 18); o += (char)(0x80 | ((cp >> 12) & 0x3f)); o += (char)(0x80 | ((cp >> 6) & 0x3f)); o += (char)(0x80 | (cp & 0x3f)); }
}

// ---- TOML (the subset br-loader configurations use) --------------------------------------
class Toml {
  public:
    explicit Toml(const std::string &t) : t_(t) {}
    Node parse()
    {
        Node root;
        root.kind = Node::Obj;
        Node *cur = &root;
        for (;;) {
            skip_ws_nl();
            if (p_ >= t_.size()) break;
            if (t_[p_] == '[') {
                bool aot = p_ + 1 < t_.size() && t_[p_ + 1] == '[';
                p_ += aot ? 2 : 1;
                skip_ws();
                std::string k = key();
                skip_ws();
                if (!eat(']') || (aot && !eat(']'))) fail("expected ']' after table name");
                end_line();
                Node *slot = root.get_mut(k);
                if (aot) {
                    if (!slot) {
                        root.obj.push_back({k, Node()});
                        slot = &root.obj.back().second;
                        slot->kind = Node::Arr;
                    } else if (slot->kind != Node::Arr) {
                        fail("cannot redefine '" + k + "' as an array of tables");
                    }
                    Node tab;
                    tab.kind = Node::Obj;
                    slot->arr.push_back(tab);
                    cur = &slot->arr.back();
                } else {
                    if (slot) fail("cannot redefine table '" + k + "'");
                    root.obj.push_back({k, Node()});
                    cur = &root.obj.back().second;
                    cur->kind = Node::Obj;
                }
                continue;
            }
            std::string k = key();
            skip_ws();
            if (!eat('=')) fail("expected '=' after key '" + k + "'");
            skip_ws();
            Node v = value();
            if (cur->get(k)) fail("cannot redefine existing key '" + k + "'");
            cur->obj.push_back({k, std::move(v)});
            end_line();
        }
        return root;
    }

  private:
    [[noreturn]] void fail(const std::string &m)
    {
        size_t line = 1, col = 1;
        for (size_t i = 0; i < p_ && i < t_.size(); ++i) {
            if (t_[i] == '\n') { ++line; col = 1; } else ++col;
        }
        throw ParseError(fmt("Error while parsing: %s\n\t(line %zu, column %zu)", m.c_str(), line, col));
    }
    bool eat(char c)
    {
        if (p_ < t_.size() && t_[p_] == c) { ++p_; return true; }
        return false;
    }
    void skip_ws()
    {
        while (p_ < t_.size() && (t_[p_] == ' ' || t_[p_] == '\t')) ++p_;
    }
    void skip_comment()
    {
        if (p_ < t_.size() && t_[p_] == '#')
            while (p_ < t_.size() && t_[p_] != '\n') ++p_;
    }
    void skip_ws_nl()   // whitespace, newlines and comments
    {
        for (;;) {
            skip_ws();
            skip_comment();
            if (p_ < t_.size() && (t_[p_] == '\n' || t_[p_] == '\r')) { ++p_; continue; }
            break;
        }
    }
    void end_line()
    {
        skip_ws();
        skip_comment();
        if (p_ < t_.size() && t_[p_] == '\r') ++p_;
        if (p_ < t_.size() && t_[p_] != '\n') fail("expected a newline after the value");
    }
    std::string key()
    {
        if (p_ < t_.size() && (t_[p_] == '"' || t_[p_] == '\'')) return str();
        size_t s = p_;
        while (p_ < t_.size() && (isalnum((unsigned char)t_[p_]) || t_[p_] == '_' || t_[p_] == '-')) ++p_;
        if (p_ == s) fail("expected a key");
        if (p_ < t_.size() && t_[p_] == '.') fail("dotted keys are not supported");
        return t_.substr(s, p_ - s);
    }
    std::string str()
    {
        char q = t_[p_++];
        std::string o;
        while (p_ < t_.size() && t_[p_] != q) {
            char c = t_[p_++];
            if (c == '\n') fail("unterminated string");
            if (q == '"' && c == '\\') {
                if (p_ >= t_.size()) break;
                char e = t_[p_++];
                switch (e) {
                case 'n': o += '\n'; break;
                case 't': o += '\t'; break;
                case 'r': o += '\r'; break;
                case 'b': o += '\b'; break;
                case 'f': o += '\f'; break;
                case '"': o += '"'; break;
                case '\\': o += '\\'; break;
                case 'u':
                case 'U': {
                    int nd = e == 'u' ? 4 : 8;
                    if (p_ + nd > t_.size()) fail("bad unicode escape");
                    unsigned cp = (unsigned)strtoul(t_.substr(p_, nd).c_str(), nullptr, 16);
                    p_ += nd;
                    put_utf8(o, cp);
                    break;
                }
                default: fail(std::string("unknown escape sequence '\\") + e + "'");
                }
            } else {
                o += c;
            }
        }
        if (!eat(q)) fail("unterminated string");
        return o;
    }
    Node value()
    {
        Node v;
        if (p_ >= t_.size()) fail("expected a value");
        char c = t_[p_];
        if (c == '"' || c == '\'') {
            v.kind = Node::Str;
            v.s = str();
        } else if (c == '[') {
            ++p_;
            v.kind = Node::Arr;
            for (;;) {
                skip_ws_nl();
                if (eat(']')) break;
                v.arr.push_back(value());
                skip_ws_nl();
                if (eat(',')) continue;
                if (eat(']')) break;
                fail("expected ',' or ']' in array");
            }
        } else if (c == '{') {
            ++p_;
            v.kind = Node::Obj;
            skip_ws();
            if (!eat('}')) {
                for (;;) {
                    skip_ws();
                    std::string k = key();
                    skip_ws();
                    if (!eat('=')) fail("expected '=' in inline table");
                    skip_ws();
                    if (v.get(k)) fail("cannot redefine existing key '" + k + "'");
                    v.obj.push_back({k, value()});
                    skip_ws();
                    if (eat(',')) continue;
                    if (eat('}')) break;
                    fail("expected ',' or '}' in inline table");
                }
            }
        } else if (t_.compare(p_, 4, "true") == 0) {
            p_ += 4;
            v.kind = Node::Bool;
            v.b = true;
        } else if (t_.compare(p_, 5, "false") == 0) {
            p_ += 5;
            v.kind = Node::Bool;
        } else {
            size_t s = p_;
            while (p_ < t_.size() && (isalnum((unsigned char)t_[p_]) || strchr("+-_.:", t_[p_]))) ++p_;
            std::string tok = t_.substr(s, p_ - s);
            std::string clean;
            for (char ch : tok)
                if (ch != '_') clean += ch;
            if (clean.empty()) fail("expected a value");
            char *end = nullptr;
            errno = 0;
            long long iv = strtoll(clean.c_str(), &end, 0);
            if (end && *end == 0 && errno == 0 && !(clean.size() > 1 && clean[0] == '0' && isdigit((unsigned char)clean[1]))) {
                v.kind = Node::Int;
                v.i = iv;
            } else {
                double dv = strtod(clean.c_str(), &end);
                if (!end || *end) fail("invalid value '" + tok + "'");
                v.kind = Node::Float;
                v.d = dv;
            }
        }
        return v;
    }
    const std::string &t_;
    size_t p_ = 0;
};

// ---- JSON -------------------------------------------------------------------------------
class Json {
  public:
    explicit Json(const std::string &t) : t_(t) {}
    Node parse()
    {
        Node v = value();
        ws();
        if (p_ != t_.size()) fail("extra data");
        return v;
    }

  private:
    [[noreturn]] void fail(const char *m) { throw ParseError(fmt("%s (offset %zu)", m, p_)); }
    void ws()
    {
        while (p_ < t_.size() && strchr(" \t\r\n", t_[p_])) ++p_;
    }
    Node value()
    {
        ws();
        if (p_ >= t_.size()) fail("unexpected end of input");
        Node v;
        char c = t_[p_];
        if (c == '{') {
            ++p_;
            v.kind = Node::Obj;
            ws();
            if (p_ < t_.size() && t_[p_] == '}') { ++p_; return v; }
            for (;;) {
                ws();
                if (p_ >= t_.size() || t_[p_] != '"') fail("expected a string key");
                std::string k = string();
                ws();
                if (p_ >= t_.size() || t_[p_++] != ':') fail("expected ':'");
                v.obj.push_back({k, value()});
                ws();
                if (p_ < t_.size() && t_[p_] == ',') { ++p_; continue; }
                if (p_ < t_.size() && t_[p_] == '}') { ++p_; break; }
                fail("expected ',' or '}'");
            }
        } else if (c == '[') {
            ++p_;
            v.kind = Node::Arr;
            ws();
            if (p_ < t_.size() && t_[p_] == ']') { ++p_; return v; }
            for (;;) {
                v.arr.push_back(value());
                ws();
                if (p_ < t_.size() && t_[p_] == ',') { ++p_; continue; }
                if (p_ < t_.size() && t_[p_] == ']') { ++p_; break; }
                fail("expected ',' or ']'");
            }
        } else if (c == '"') {
            v.kind = Node::Str;
            v.s = string();
        } else if (t_.compare(p_, 4, "true") == 0) {
            p_ += 4;
            v.kind = Node::Bool;
            v.b = true;
        } else if (t_.compare(p_, 5, "false") == 0) {
            p_ += 5;
            v.kind = Node::Bool;
        } else if (t_.compare(p_, 4, "null") == 0) {
            p_ += 4;
        } else {
            size_t s = p_;
            while (p_ < t_.size() && strchr("+-0123456789.eE", t_[p_])) ++p_;
            if (p_ == s) fail("syntax error");
            std::string tok = t_.substr(s, p_ - s);
            char *end = nullptr;
            if (tok.find_first_of(".eE") == std::string::npos) {
                v.kind = Node::Int;
                v.i = strtoll(tok.c_str(), &end, 10);
            } else {
                v.kind = Node::Float;
                v.d = strtod(tok.c_str(), &end);
            }
            if (!end || *end) fail("bad number");
        }
        return v;
    }
    std::string string()
    {
        ++p_;
        std::string o;
        while (p_ < t_.size() && t_[p_] != '"') {
            char c = t_[p_++];
            if (c != '\\') { o += c; continue; }
            if (p_ >= t_.size()) break;
            char e = t_[p_++];
            switch (e) {
            case 'n': o += '\n'; break;
            case 't': o += '\t'; break;
            case 'r': o += '\r'; break;
            case 'b': o += '\b'; break;
            case 'f': o += '\f'; break;
            case '/': o += '/'; break;
            case '"': o += '"'; break;
            case '\\': o += '\\'; break;
            case 'u':
                if (p_ + 4 > t_.size()) fail("bad escape");
                put_utf8(o, (unsigned)strtoul(t_.substr(p_, 4).c_str(), nullptr, 16));
                p_ += 4;
                break;
            default: fail("bad escape");
            }
        }
        if (p_ >= t_.size()) fail("unterminated string");
        ++p_;
        return o;
    }
    const std::string &t_;
    size_t p_ = 0;
};

// ---- the configuration model (config.hpp) -----------------------------------------------
struct Ip {
    int family = 0;   // AF_INET / AF_INET6
    uint8_t a[16] = {0};
    bool operator==(const Ip &o) const { return family == o.family && memcmp(a, o.a, 16) == 0; }
    std::string str() const
    {
        char buf[INET6_ADDRSTRLEN] = {0};
        inet_ntop(family, a, buf, sizeof buf);
        return buf;
    }
};
struct UdpEp {
    Ip ip;
    uint16_t port = 0;
    std::string str() const { return "[" + ip.str() + "]:" + std::to_string(port); }
};
struct ExternalIface { uint32_t ifid; std::string ifname; UdpEp local, remote; };
struct SiblingIface { uint32_t ifid; UdpEp sibling; };
struct InternalIface { std::string ifname; UdpEp local; };
struct BrSetup {
    std::string self;
    std::vector<ExternalIface> external;
    std::vector<SiblingIface> sibling;
    std::vector<InternalIface> internal;
};

static bool parse_ip(const std::string &s, Ip *out)
{
    Ip ip;
    if (inet_pton(AF_INET, s.c_str(), ip.a) == 1) ip.family = AF_INET;
    else if (inet_pton(AF_INET6, s.c_str(), ip.a) == 1) ip.family = AF_INET6;
    else return false;
    *out = ip;
    return true;
}

// parseUdpEp (config.cpp:66-90): "127.0.0.1:50000" or "[::1]:50000"
static UdpEp parse_udp_ep(const std::string &s)
{
    size_t pos = s.rfind(':');
    if (pos == std::string::npos) throw std::invalid_argument("Invalid underlay address");
    std::string ip = s.substr(0, pos), port = s.substr(pos + 1);
    if (!ip.empty() && ip.front() == '[') ip.erase(0, 1);
    if (!ip.empty() && ip.back() == ']') ip.pop_back();
    UdpEp ep;
    if (!parse_ip(ip, &ep.ip)) throw std::invalid_argument("Invalid argument: " + ip);
    // boost::lexical_cast<uint16_t>
    bool ok = !port.empty() && port.size() <= 5;
    for (char c : port) ok = ok && isdigit((unsigned char)c);
    if (!ok || atol(port.c_str()) > 0xffff)
        throw std::invalid_argument("bad lexical cast: source type value could not be interpreted as target");
    ep.port = (uint16_t)atol(port.c_str());
    return ep;
}

static uint32_t parse_ifid(const std::string &k)
{
    bool ok = !k.empty() && k.size() <= 10;
    for (char c : k) ok = ok && isdigit((unsigned char)c);
    if (!ok || strtoull(k.c_str(), nullptr, 10) > 0xffffffffull)
        throw std::invalid_argument("bad lexical cast: source type value could not be interpreted as target");
    return (uint32_t)strtoul(k.c_str(), nullptr, 10);
}

static const Node &at(const Node &n, const char *k)
{
    if (n.kind != Node::Obj) throw std::invalid_argument("not an object");
    const Node *v = n.get(k);
    if (!v) throw std::out_of_range(std::string("key not found: ") + k);
    return *v;
}

static const std::string &as_string(const Node &n)
{
    if (n.kind != Node::Str) throw std::invalid_argument("not a string");
    return n.s;
}

// parseTopology (config.cpp:97-140)
static void parse_topology(const Node &topo, const std::string &self, BrSetup &setup)
{
    const Node &brs = at(topo, "border_routers");
    if (brs.kind != Node::Obj) throw std::invalid_argument("not an object");
    for (const auto &br : brs.obj) {
        const Node &ifaces = at(br.second, "interfaces");
        if (ifaces.kind != Node::Obj) throw std::invalid_argument("not an object");
        if (br.first == self) {
            for (const auto &iface : ifaces.obj) {
                const Node &underlay = at(iface.second, "underlay");
                uint32_t ifid = parse_ifid(iface.first);
                UdpEp local = parse_udp_ep(as_string(at(underlay, "public")));
                UdpEp remote = parse_udp_ep(as_string(at(underlay, "remote")));
                if (local.ip.family != remote.ip.family)
                    throw std::invalid_argument(
                        "Local and remote addresses of a SCION link must be of the same IP version.");
                setup.external.push_back({ifid, "", local, remote});
            }
        } else {
            UdpEp sib = parse_udp_ep(as_string(at(br.second, "internal_addr")));
            for (const auto &iface : ifaces.obj) setup.sibling.push_back({parse_ifid(iface.first), sib});
        }
    }
}

// parseInternalIfaces (config.cpp:147-170)
static void parse_internal(const Node &conf, BrSetup &setup)
{
    const Node *ifaces = conf.get("internal_interfaces");
    bool ok = ifaces && ifaces->kind == Node::Arr;
    for (size_t i = 0; ok && i < ifaces->arr.size(); ++i) ok = ifaces->arr[i].kind == Node::Obj;
    if (!ok) throw std::invalid_argument("Configuration item 'internal_interfaces' is missing or has an invalid value.");
    for (const Node &t : ifaces->arr) {
        const Node *ip = t.get("ip");
        if (!ip || ip->kind != Node::Str) throw std::invalid_argument("Internal interface is missing an IP address.");
        const Node *port = t.get("port");
        if (!port || port->kind != Node::Int || port->i < 0 || port->i > 0xffff)
            throw std::invalid_argument("Internal interface is missing the UDP port.");
        InternalIface iface;
        if (!parse_ip(ip->s, &iface.local.ip)) throw std::invalid_argument("Invalid argument: " + ip->s);
        iface.local.port = (uint16_t)port->i;
        setup.internal.push_back(iface);
    }
}

static bool read_file(const char *path, std::string *out)
{
    FILE *f = fopen(path, "rb");
    if (!f) return false;
    char buf[65536];
    size_t n;
    out->clear();
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) out->append(buf, n);
    fclose(f);
    return true;
}

struct IfAddr {
    Ip ip;
    std::string name;
    uint32_t ifindex;
};

// getIfAddr (config.cpp:168-204): this network namespace's addresses
static std::vector<IfAddr> system_if_addrs()
{
    std::vector<IfAddr> out;
    ifaddrs *ifa = nullptr;
    if (getifaddrs(&ifa) != 0) return out;
    for (ifaddrs *p = ifa; p; p = p->ifa_next) {
        if (!p->ifa_addr) continue;
        IfAddr e;
        if (p->ifa_addr->sa_family == AF_INET) {
            e.ip.family = AF_INET;
            memcpy(e.ip.a, &reinterpret_cast<sockaddr_in *>(p->ifa_addr)->sin_addr, 4);
        } else if (p->ifa_addr->sa_family == AF_INET6) {
            e.ip.family = AF_INET6;
            memcpy(e.ip.a, &reinterpret_cast<sockaddr_in6 *>(p->ifa_addr)->sin6_addr, 16);
        } else {
            continue;
        }
        e.name = p->ifa_name;
        e.ifindex = if_nametoindex(p->ifa_name);
        out.push_back(e);
    }
    freeifaddrs(ifa);
    return out;
}

static const IfAddr *find_addr(const std::vector<IfAddr> &v, const Ip &ip)
{
    const IfAddr *hit = nullptr;   // the map is filled in order: the last entry for an address wins
    for (const auto &e : v)
        if (e.ip == ip) hit = &e;
    return hit;
}

static void put(std::string *o, const std::string &s)
{
    if (o) *o += s;
}

// loadConfig (config.cpp:212-262).  Returns false after writing br-loader's diagnostics.
static bool load_config(const char *path, const std::vector<IfAddr> &ifmap, BrSetup *setup, std::string *diag)
{
    std::string text;
    Node conf;
    if (!read_file(path, &text)) {
        put(diag, fmt("Parsing configuration failed:\nFile could not be opened for reading\n\t(in '%s')\n", path));
        return false;
    }
    try {
        conf = Toml(text).parse();
    } catch (const ParseError &e) {
        put(diag, std::string("Parsing configuration failed:\n") + e.what() + fmt("\n\t(in '%s')\n", path));
        return false;
    }
    const Node *self = conf.get("self");
    if (!self || self->kind != Node::Str) {
        put(diag, "Configuration item 'self' is missing or has an invalid value.\n");
        return false;
    }
    setup->self = self->s;
    const Node *topo_file = conf.get("topology");
    if (!topo_file || topo_file->kind != Node::Str) {
        put(diag, "Configuration item 'topology' is missing or has an invalid value.\n");
        return false;
    }
    std::string topo_text;
    if (!read_file(topo_file->s.c_str(), &topo_text)) {
        put(diag, "File not found: " + topo_file->s + "\n");
        return false;
    }
    try {
        parse_topology(Json(topo_text).parse(), setup->self, *setup);
    } catch (const std::exception &e) {
        put(diag, std::string("Parsing topology file failed:\n") + e.what() + "\n");
        return false;
    }
    try {
        parse_internal(conf, *setup);
    } catch (const std::exception &e) {
        put(diag, std::string(e.what()) + "\n");
        return false;
    }
    for (auto &i : setup->external) {
        const IfAddr *a = find_addr(ifmap, i.local.ip);
        if (a) i.ifname = a->name;
        else put(diag, fmt("WARNING: No interface has IP %s\n         Cannot forward packets to IFID %u\n",
                           i.local.ip.str().c_str(), i.ifid));
    }
    for (auto &i : setup->internal) {
        const IfAddr *a = find_addr(ifmap, i.local.ip);
        if (a) i.ifname = a->name;
        else put(diag, fmt("WARNING: No interface has IP %s\n", i.local.ip.str().c_str()));
    }
    return true;
}

// operator<< (config.cpp:296-330)
static std::string listing(const BrSetup &s)
{
    std::string o = "XDP Border Router " + s.self + "\nExternal interfaces:\n";
    for (const auto &i : s.external) {
        o += fmt("%5u %6s local  %s\n", i.ifid, i.ifname.c_str(), i.local.str().c_str());
        o += fmt("             remote %s\n", i.remote.str().c_str());
    }
    o += "Sibling BR interfaces:\n";
    for (const auto &i : s.sibling) o += fmt("%5u route to %s\n", i.ifid, i.sibling.str().c_str());
    o += "Internal interfaces:\n";
    for (const auto &i : s.internal) o += fmt("%6s %s\n", i.ifname.c_str(), i.local.str().c_str());
    return o;
}

static uint32_t fam(const Ip &ip) { return ip.family == AF_INET ? HFV_AF_INET : HFV_AF_INET6; }
static void be16(uint8_t out[2], uint16_t v) { out[0] = (uint8_t)(v >> 8); out[1] = (uint8_t)v; }

static uint32_t ifindex_of(const std::vector<IfAddr> &ifmap, const std::string &name)
{
    for (const auto &e : ifmap)
        if (e.name == name) return e.ifindex;
    return if_nametoindex(name.c_str());   // ifNameToIndex (ifindex.cpp)
}

// initializeMaps' table fills (maps.cpp:91-200) into one hfv_br_config.  Maps keyed by
// ifindex / ifid keep the last update for a key, like the BPF map updates.
static int build_tables(const BrSetup &s, const std::vector<IfAddr> &ifmap, const hfv_br_next_hop *hops, size_t n_hops,
                        hfv_br_config *cfg, std::string *diag)
{
    memset(cfg, 0, sizeof *cfg);
    auto full = [&](const char *what) {
        put(diag, fmt("too many %s for the router tables (%d interfaces, %d routes, %d tx ports)\n", what,
                      HFV_BR_MAX_IFACES, HFV_BR_MAX_ROUTES, HFV_BR_MAX_TXPORTS));
        return -ENOSPC;
    };
    for (const auto &i : s.external) {   // populateIngressMap: {local ip, port, ifindex} -> ifid
        if (i.ifname.empty()) continue;
        if (cfg->n_ingress >= HFV_BR_MAX_IFACES) return full("ingress interfaces");
        hfv_br_ingress &e = cfg->ingress[cfg->n_ingress++];
        e.ifindex = ifindex_of(ifmap, i.ifname);
        e.family = fam(i.local.ip);
        memcpy(e.addr, i.local.ip.a, 16);
        be16(e.port, i.local.port);
        e.ifid = i.ifid;
    }
    auto egress_slot = [&](uint32_t ifid) -> hfv_br_egress * {   // populateEgressMap: ifid -> fwd_info
        for (uint32_t k = 0; k < cfg->n_egress; ++k)
            if (cfg->egress[k].ifid == ifid) return &cfg->egress[k];
        if (cfg->n_egress >= HFV_BR_MAX_IFACES) return nullptr;
        return &cfg->egress[cfg->n_egress++];
    };
    for (const auto &i : s.external) {
        hfv_br_egress *e = egress_slot(i.ifid);
        if (!e) return full("egress interfaces");
        memset(e, 0, sizeof *e);
        e->ifid = i.ifid;
        e->fwd_external = 1;
        e->family = fam(i.remote.ip);
        memcpy(e->remote, i.remote.ip.a, 16);
        memcpy(e->local, i.local.ip.a, 16);
        be16(e->remote_port, i.remote.port);
        be16(e->local_port, i.local.port);
    }
    for (const auto &i : s.sibling) {
        hfv_br_egress *e = egress_slot(i.ifid);
        if (!e) return full("egress interfaces");
        memset(e, 0, sizeof *e);
        e->ifid = i.ifid;
        e->family = fam(i.sibling.ip);
        memcpy(e->remote, i.sibling.ip.a, 16);
        be16(e->remote_port, i.sibling.port);
    }
    for (const auto &i : s.internal) {   // populateIntIfMap: ifindex -> internal address
        if (i.ifname.empty()) continue;
        uint32_t ifx = ifindex_of(ifmap, i.ifname);
        hfv_br_int_iface *e = nullptr;
        for (uint32_t k = 0; k < cfg->n_int_ifaces; ++k)
            if (cfg->int_ifaces[k].ifindex == ifx) e = &cfg->int_ifaces[k];
        if (!e) {
            if (cfg->n_int_ifaces >= HFV_BR_MAX_IFACES) return full("internal interfaces");
            e = &cfg->int_ifaces[cfg->n_int_ifaces++];
        }
        memset(e, 0, sizeof *e);
        e->ifindex = ifx;
        e->family = fam(i.local.ip);
        memcpy(e->addr, i.local.ip.a, 16);
        be16(e->port, i.local.port);
    }
    auto tx = [&](const std::string &ifname) {   // populatePortMap: the devmap of redirect targets
        uint32_t ifx = ifindex_of(ifmap, ifname);
        for (uint32_t k = 0; k < cfg->n_tx_ports; ++k)
            if (cfg->tx_ports[k] == ifx) return 0;
        if (cfg->n_tx_ports >= HFV_BR_MAX_TXPORTS) return -1;
        cfg->tx_ports[cfg->n_tx_ports++] = ifx;
        return 0;
    };
    for (const auto &i : s.external)
        if (!i.ifname.empty() && tx(i.ifname)) return full("tx ports");
    for (const auto &i : s.internal)
        if (!i.ifname.empty() && tx(i.ifname)) return full("tx ports");
    for (size_t k = 0; k < n_hops; ++k) {   // the static FIB (replaces bpf_fib_lookup)
        if (cfg->n_routes >= HFV_BR_MAX_ROUTES) return full("routes");
        const hfv_br_next_hop &h = hops[k];
        hfv_br_route &r = cfg->routes[cfg->n_routes++];
        r.family = h.family;
        memcpy(r.prefix, h.prefix, 16);
        r.prefix_len = h.prefix_len;
        r.ret = h.ret;
        char name[sizeof h.ifname + 1] = {0};
        memcpy(name, h.ifname, sizeof h.ifname);
        r.ifindex = ifindex_of(ifmap, name);
        memcpy(r.smac, h.smac, 6);
        memcpy(r.dmac, h.dmac, 6);
    }
    return 0;
}

static void copy_out(const std::string &s, char *buf, size_t len)
{
    if (!buf || !len) return;
    size_t n = s.size() < len - 1 ? s.size() : len - 1;
    memcpy(buf, s.data(), n);
    buf[n] = 0;
}

// ---- pinned router tables ($HFV_PIN_DIR/<br>/br_config) -----------------------------------
struct BrcfgFile {
    char magic[8];
    uint32_t version;
    uint32_t seq;          // seqlock: odd while a writer updates the tables
    uint32_t detached;     // 1: `hfv-loader detach` -- attached data planes pass every frame
    uint32_t feat_off;     // HFV_BR_NO_*: build options the attached router runs without
    uint8_t reserved[40];
    hfv_br_config cfg;
};
static_assert(sizeof(BrcfgFile) == 64 + sizeof(hfv_br_config), "pinned file layout unchanged");
static const char kBrMagic[8] = {'H', 'F', 'V', 'B', 'R', 'C', 'F', '1'};

static int mkdir_parents(const char *path)
{
    char tmp[4096];
    if (strlen(path) >= sizeof tmp) return -ENAMETOOLONG;
    strcpy(tmp, path);
    for (char *p = tmp + 1; *p; ++p) {
        if (*p != '/') continue;
        *p = 0;
        if (mkdir(tmp, 0755) != 0 && errno != EEXIST) return -errno;
        *p = '/';
    }
    return 0;
}

}  // namespace

// Consistent snapshot of a pinned br_config mapping (tables and detached flag); returns its
// (even) seq.
uint32_t brcfg_snapshot(const void *mapping, hfv_br_config *out, uint32_t *detached, uint32_t *feat_off)
{
    const BrcfgFile *f = (const BrcfgFile *)mapping;
    for (;;) {
        uint32_t s0 = __atomic_load_n(&f->seq, __ATOMIC_ACQUIRE);
        if (s0 & 1u) { usleep(10); continue; }
        memcpy(out, &f->cfg, sizeof *out);
        const uint32_t d = __atomic_load_n(&f->detached, __ATOMIC_RELAXED);
        const uint32_t fo = __atomic_load_n(&f->feat_off, __ATOMIC_RELAXED);
        std::atomic_thread_fence(std::memory_order_acquire);
        if (__atomic_load_n(&f->seq, __ATOMIC_ACQUIRE) == s0) {
            if (detached) *detached = d;
            if (feat_off) *feat_off = fo;
            return s0;
        }
    }
}

// Table counts within the fixed capacity of struct hfv_br_config / DevBrConfig: the compile
// loops index the arrays by them, so a snapshot of a stale, foreign or corrupt pinned file is
// checked before it is used.
int br_config_check(const hfv_br_config *cfg)
{
    if (cfg->n_int_ifaces > HFV_BR_MAX_IFACES || cfg->n_ingress > HFV_BR_MAX_IFACES ||
        cfg->n_egress > HFV_BR_MAX_IFACES || cfg->n_routes > HFV_BR_MAX_ROUTES || cfg->n_tx_ports > HFV_BR_MAX_TXPORTS)
        return -EINVAL;
    return 0;
}
uint32_t brcfg_seq(const void *mapping) { return __atomic_load_n(&((const BrcfgFile *)mapping)->seq, __ATOMIC_ACQUIRE); }

int brcfg_open_ro(const char *path, const void **mapping)
{
    int fd = open(path, O_RDONLY);
    if (fd < 0) return -errno;
    struct stat st;
    if (fstat(fd, &st) != 0 || (size_t)st.st_size != sizeof(BrcfgFile)) { close(fd); return -EINVAL; }
    void *m = mmap(nullptr, sizeof(BrcfgFile), PROT_READ, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) return -errno;
    if (memcmp(((const BrcfgFile *)m)->magic, kBrMagic, 8) != 0) { munmap(m, sizeof(BrcfgFile)); return -EINVAL; }
    *mapping = m;
    return 0;
}
void brcfg_close(const void *mapping)
{
    if (mapping) munmap((void *)mapping, sizeof(BrcfgFile));
}

}  // namespace hfv

using namespace hfv;

extern "C" {

int hfv_br_config_load(const char *toml_path, const struct hfv_br_ifaddr *ifaddrs, size_t n_ifaddrs,
                       const struct hfv_br_next_hop *hops, size_t n_hops, struct hfv_br_config *out, char *self,
                       size_t self_len, char *listing_buf, size_t listing_len, char *diag_buf, size_t diag_len)
{
    if (!toml_path || !out || (!hops && n_hops) || (!ifaddrs && n_ifaddrs)) return fail(-EINVAL, "null argument");
    std::vector<IfAddr> ifmap;
    if (ifaddrs) {
        for (size_t k = 0; k < n_ifaddrs; ++k) {
            IfAddr e;
            e.ip.family = ifaddrs[k].family == HFV_AF_INET ? AF_INET : AF_INET6;
            memcpy(e.ip.a, ifaddrs[k].addr, 16);
            char name[sizeof ifaddrs[k].ifname + 1] = {0};
            memcpy(name, ifaddrs[k].ifname, sizeof ifaddrs[k].ifname);
            e.name = name;
            e.ifindex = ifaddrs[k].ifindex;
            ifmap.push_back(e);
        }
    } else {
        ifmap = system_if_addrs();
    }
    BrSetup setup;
    std::string diag;
    if (!load_config(toml_path, ifmap, &setup, &diag)) {
        copy_out(diag, diag_buf, diag_len);
        std::string first = diag.substr(0, diag.find('\n'));
        return fail(-EINVAL, "%s: %s", toml_path, first.c_str());
    }
    int rc = build_tables(setup, ifmap, hops, n_hops, out, &diag);
    copy_out(diag, diag_buf, diag_len);
    copy_out(setup.self, self, self_len);
    copy_out(listing(setup), listing_buf, listing_len);
    if (rc) return fail(rc, "%s: router tables overflow", toml_path);
    return 0;
}

int hfv_brconfig_path(const char *br, char *out, size_t len)
{
    if (!br || !out || !*br || strchr(br, '/')) return fail(-EINVAL, "invalid BR name");
    const char *base = getenv("HFV_PIN_DIR");
    if (!base || !*base) base = "/dev/shm/hfv";
    int w = snprintf(out, len, "%s/%s/br_config", base, br);
    if (w < 0 || (size_t)w >= len) return fail(-ENAMETOOLONG, "path too long");
    return 0;
}

int hfv_brconfig_publish(const char *path, const struct hfv_br_config *cfg)
{
    return hfv_brconfig_publish_opts(path, cfg, 0);
}

int hfv_br_config_check_options(const struct hfv_br_config *cfg, uint32_t disabled)
{
    if (!cfg) return fail(-EINVAL, "null argument");
    if (disabled & ~(HFV_BR_NO_IPV4 | HFV_BR_NO_IPV6 | HFV_BR_NO_SCION_PATH)) return fail(-EINVAL, "unknown build option");
    if (br_config_check(cfg)) return fail(-EINVAL, "router table larger than the fixed capacity");
    // the tables initializeMaps stores addresses into (maps.cpp:91-200): ingress keys, links and
    // siblings, internal interfaces
    auto off = [&](uint32_t family) {
        return (family == HFV_AF_INET && (disabled & HFV_BR_NO_IPV4)) || (family == HFV_AF_INET6 && (disabled & HFV_BR_NO_IPV6));
    };
    bool bad4 = false, bad6 = false;
    auto note = [&](uint32_t family) {
        if (off(family)) (family == HFV_AF_INET ? bad4 : bad6) = true;
    };
    for (uint32_t i = 0; i < cfg->n_ingress; ++i) note(cfg->ingress[i].family);
    for (uint32_t i = 0; i < cfg->n_egress; ++i) note(cfg->egress[i].family);
    for (uint32_t i = 0; i < cfg->n_int_ifaces; ++i) note(cfg->int_ifaces[i].family);
    if (bad4) return fail(-EINVAL, "Border router configuration contains IPv4 address, but IPv4 support is deactivated.");
    if (bad6) return fail(-EINVAL, "Border router configuration contains IPv6 address, but IPv6 support is deactivated.");
    return 0;
}

int hfv_brconfig_publish_opts(const char *path, const struct hfv_br_config *cfg, uint32_t disabled)
{
    if (!path || !cfg) return fail(-EINVAL, "null argument");
    if (hfv_br_config_check_options(cfg, disabled)) return -EINVAL;
    if (br_config_check(cfg))
        return fail(-EINVAL, "router table larger than the fixed capacity (%d interfaces, %d routes, %d tx ports)",
                    HFV_BR_MAX_IFACES, HFV_BR_MAX_ROUTES, HFV_BR_MAX_TXPORTS);
    int rc = mkdir_parents(path);
    if (rc) return fail(rc, "cannot create the directory of %s", path);
    int fd = open(path, O_RDWR | O_CREAT, 0644);
    if (fd < 0) return fail(-errno, "cannot open %s", path);
    if (flock(fd, LOCK_EX) != 0) { int e = -errno; close(fd); return fail(e, "flock %s", path); }
    struct stat st;
    if (fstat(fd, &st) != 0 || (st.st_size != 0 && (size_t)st.st_size != sizeof(BrcfgFile)) ||
        (st.st_size == 0 && ftruncate(fd, sizeof(BrcfgFile)) != 0)) {
        close(fd);
        return fail(-EINVAL, "%s is not a pinned router config", path);
    }
    void *m = mmap(nullptr, sizeof(BrcfgFile), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (m == MAP_FAILED) { int e = -errno; close(fd); return fail(e, "mmap %s", path); }
    BrcfgFile *f = (BrcfgFile *)m;
    if (memcmp(f->magic, kBrMagic, 8) != 0) {
        if (st.st_size != 0 && f->magic[0] != 0) {
            munmap(m, sizeof(BrcfgFile));
            close(fd);
            return fail(-EINVAL, "%s is not a pinned router config", path);
        }
        memcpy(f->magic, kBrMagic, 8);
        f->version = 1;
    }
    __atomic_store_n(&f->seq, f->seq + 1, __ATOMIC_RELAXED);   // odd: update in progress
    std::atomic_thread_fence(std::memory_order_release);
    f->cfg = *cfg;
    __atomic_store_n(&f->detached, 0u, __ATOMIC_RELAXED);
    __atomic_store_n(&f->feat_off, disabled, __ATOMIC_RELAXED);
    __atomic_store_n(&f->seq, f->seq + 1, __ATOMIC_RELEASE);   // even: published
    msync(m, sizeof(BrcfgFile), MS_SYNC);
    munmap(m, sizeof(BrcfgFile));
    close(fd);
    return 0;
}

int hfv_brconfig_detach(const char *path)
{
    if (!path) return fail(-EINVAL, "null argument");
    int fd = open(path, O_RDWR);
    if (fd < 0) return fail(-ENOENT, "not attached: %s", path);
    if (flock(fd, LOCK_EX) != 0) { int e = -errno; close(fd); return fail(e, "flock %s", path); }
    struct stat st;
    void *m = MAP_FAILED;
    if (fstat(fd, &st) == 0 && (size_t)st.st_size == sizeof(BrcfgFile))
        m = mmap(nullptr, sizeof(BrcfgFile), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (m == MAP_FAILED || memcmp(((BrcfgFile *)m)->magic, kBrMagic, 8) != 0) {
        if (m != MAP_FAILED) munmap(m, sizeof(BrcfgFile));
        close(fd);
        return fail(-EINVAL, "%s is not a pinned router config", path);
    }
    BrcfgFile *f = (BrcfgFile *)m;
    int rc = 0;
    if (__atomic_load_n(&f->detached, __ATOMIC_RELAXED)) {
        rc = fail(-ENOENT, "not attached: %s", path);
    } else {
        // the file stays (attached data planes keep their mapping of this inode and see the
        // flag at their next batch; a later attach republishes into the same file)
        __atomic_store_n(&f->seq, f->seq + 1, __ATOMIC_RELAXED);
        std::atomic_thread_fence(std::memory_order_release);
        __atomic_store_n(&f->detached, 1u, __ATOMIC_RELAXED);
        __atomic_store_n(&f->seq, f->seq + 1, __ATOMIC_RELEASE);
        msync(m, sizeof(BrcfgFile), MS_SYNC);
    }
    munmap(m, sizeof(BrcfgFile));
    close(fd);
    return rc;
}

int hfv_brconfig_read(const char *path, struct hfv_br_config *cfg)
{
    if (!path || !cfg) return fail(-EINVAL, "null argument");
    const void *m = nullptr;
    int rc = brcfg_open_ro(path, &m);
    if (rc) return fail(rc, "cannot open pinned router config %s", path);
    uint32_t detached = 0;
    brcfg_snapshot(m, cfg, &detached);
    brcfg_close(m);
    if (br_config_check(cfg)) return fail(-EINVAL, "pinned router config %s holds counts past the fixed capacity", path);
    if (detached) return fail(-ENOENT, "not attached: %s (detached)", path);
    return 0;
}

}  // extern "C"
