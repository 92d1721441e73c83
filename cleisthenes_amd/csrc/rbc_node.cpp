// rbc_node.cpp -- the RBC state machine and its wire codec.
//
// The reference's rbc package (rbc/rbc.go:9-100) declares the instance,
// its handlers and the three request types (rbc/request.go:9-21) but leaves
// every body unimplemented; the protocol it names is HBBFT's reliable
// broadcast (docs/RBC-EN.md).  This file implements it on top of the GPU
// data path: every shard / validateMessage / interpolate goes to an
// rbc_batcher without blocking, so the thousands of concurrent instances of
// an ACS round (one per proposer, at every node hosted by the process) share
// batched launches.  Completions are applied in submission order by
// rbc_node_progress.
#include <string.h>

#include <deque>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/rbc_protocol.h"

namespace {

// ---------------------------------------------------------------------------
// protobuf wire format (pb/message.pb.go:84-183): Message.rbc = field 3,
// RBC.payload = field 1 (bytes), RBC.type = field 2 (varint enum)
// ---------------------------------------------------------------------------
void put_varint(std::string &s, uint64_t v) {
    while (v >= 0x80) {
        s.push_back((char)(v | 0x80));
        v >>= 7;
    }
    s.push_back((char)v);
}

bool get_varint(const uint8_t *&p, const uint8_t *e, uint64_t *v) {
    uint64_t r = 0;
    for (int sh = 0; sh < 64; sh += 7) {
        if (p >= e) return false;
        const uint8_t b = *p++;
        r |= (uint64_t)(b & 0x7f) << sh;
        if (!(b & 0x80)) {
            *v = r;
            return true;
        }
    }
    return false;
}

bool get_len(const uint8_t *&p, const uint8_t *e, const uint8_t **body, size_t *n) {
    uint64_t l;
    if (!get_varint(p, e, &l) || l > (uint64_t)(e - p)) return false;
    *body = p;
    *n = (size_t)l;
    p += l;
    return true;
}

bool skip_field(const uint8_t *&p, const uint8_t *e, int wire) {
    uint64_t v;
    const uint8_t *b;
    size_t n;
    switch (wire) {
        case 0: return get_varint(p, e, &v);
        case 1:
            if (e - p < 8) return false;
            p += 8;
            return true;
        case 2: return get_len(p, e, &b, &n);
        case 5:
            if (e - p < 4) return false;
            p += 4;
            return true;
        default: return false;  // groups are not used by proto3
    }
}

size_t varint_len(uint64_t v) {
    size_t n = 1;
    while (v >= 0x80) {
        v >>= 7;
        ++n;
    }
    return n;
}

std::string pb_rbc(int type, const uint8_t *payload, size_t len) {
    // proto3: default (empty / zero) scalars are not emitted
    const size_t body = (len ? 1 + varint_len(len) + len : 0) + (type ? 1 + varint_len((uint64_t)type) : 0);
    std::string m;
    m.reserve(1 + varint_len(body) + body);
    m.push_back(0x1a);  // field 3, length-delimited: the oneof is set even when RBC is empty
    put_varint(m, body);
    if (len) {
        m.push_back(0x0a);
        put_varint(m, len);
        m.append((const char *)payload, len);
    }
    if (type) {
        m.push_back(0x10);
        put_varint(m, (uint64_t)type);
    }
    return m;
}

// Message parse with protobuf merge semantics: a repeated RBC field merges
// (later scalars win), a BBA field switches the oneof away, unknown fields
// are skipped.
int pb_parse(const uint8_t *msg, size_t len, int *type, const uint8_t **payload, size_t *payload_len) {
    const uint8_t *p = msg, *e = msg + len;
    bool is_rbc = false;
    uint64_t t = 0;
    const uint8_t *pl = nullptr;
    size_t pll = 0;
    while (p < e) {
        uint64_t key;
        if (!get_varint(p, e, &key)) return RBC_ERR_PROTOCOL;
        const int field = (int)(key >> 3), wire = (int)(key & 7);
        if (field == 0) return RBC_ERR_PROTOCOL;
        if ((field == 3 || field == 4) && wire == 2) {
            const uint8_t *body;
            size_t n;
            if (!get_len(p, e, &body, &n)) return RBC_ERR_PROTOCOL;
            if (field == 4) {
                is_rbc = false;
                t = 0;
                pl = nullptr;
                pll = 0;
                continue;
            }
            is_rbc = true;
            const uint8_t *q = body, *qe = body + n;
            while (q < qe) {
                uint64_t k2;
                if (!get_varint(q, qe, &k2)) return RBC_ERR_PROTOCOL;
                const int f2 = (int)(k2 >> 3), w2 = (int)(k2 & 7);
                if (f2 == 0) return RBC_ERR_PROTOCOL;
                if (f2 == 1 && w2 == 2) {
                    if (!get_len(q, qe, &pl, &pll)) return RBC_ERR_PROTOCOL;
                } else if (f2 == 2 && w2 == 0) {
                    if (!get_varint(q, qe, &t)) return RBC_ERR_PROTOCOL;
                } else if (!skip_field(q, qe, w2)) {
                    return RBC_ERR_PROTOCOL;
                }
            }
        } else if (!skip_field(p, e, wire)) {
            return RBC_ERR_PROTOCOL;
        }
    }
    if (!is_rbc || t > RBC_MSG_READY) return RBC_ERR_PROTOCOL;
    *type = (int)t;
    *payload = pl;
    *payload_len = pll;
    return RBC_OK;
}

// ---------------------------------------------------------------------------
// Go encoding/json for []byte (standard base64, padded) and the request structs
// ---------------------------------------------------------------------------
const char B64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

// Written straight into pre-sized storage: a VAL / ECHO carries a whole shard
// (tens of KiB) as base64, so the codec is the per-message host cost.
void b64_encode(std::string &s, const uint8_t *p, size_t n) {
    const size_t at = s.size();
    s.resize(at + 4 * ((n + 2) / 3));
    char *o = &s[at];
    size_t i = 0;
    for (; i + 3 <= n; i += 3, o += 4) {
        const uint32_t v = (uint32_t)p[i] << 16 | (uint32_t)p[i + 1] << 8 | p[i + 2];
        o[0] = B64[v >> 18];
        o[1] = B64[(v >> 12) & 63];
        o[2] = B64[(v >> 6) & 63];
        o[3] = B64[v & 63];
    }
    if (n - i == 1) {
        const uint32_t v = (uint32_t)p[i] << 16;
        o[0] = B64[v >> 18];
        o[1] = B64[(v >> 12) & 63];
        o[2] = o[3] = '=';
    } else if (n - i == 2) {
        const uint32_t v = (uint32_t)p[i] << 16 | (uint32_t)p[i + 1] << 8;
        o[0] = B64[v >> 18];
        o[1] = B64[(v >> 12) & 63];
        o[2] = B64[(v >> 6) & 63];
        o[3] = '=';
    }
}

// alphabet value of every byte, -1 outside the standard alphabet
struct B64Table {
    int8_t v[256];
    B64Table() {
        memset(v, -1, sizeof v);
        for (int i = 0; i < 64; ++i) v[(uint8_t)B64[i]] = (int8_t)i;
    }
};
const B64Table kB64;

// base64.StdEncoding.DecodeString as encoding/json applies it: padding
// required, '\r' / '\n' ignored.  StdEncoding is not Strict(), so non-zero
// trailing bits in the last quantum are ignored ("AB==" decodes to 0x00).
bool b64_decode_range(const char *in, size_t len, std::string &out) {
    std::string filtered;
    if (memchr(in, '\r', len) || memchr(in, '\n', len)) {
        filtered.reserve(len);
        for (size_t i = 0; i < len; ++i)
            if (in[i] != '\r' && in[i] != '\n') filtered.push_back(in[i]);
        in = filtered.data();
        len = filtered.size();
    }
    if (len % 4) return false;
    out.resize(len / 4 * 3);
    char *o = len ? &out[0] : nullptr;
    size_t w = 0;
    for (size_t i = 0; i < len; i += 4) {
        const uint8_t *q = reinterpret_cast<const uint8_t *>(in + i);
        int pad = 0;
        if (i + 4 == len && q[3] == '=') pad = q[2] == '=' ? 2 : 1;
        int v[4] = {0, 0, 0, 0};
        for (int j = 0; j < 4 - pad; ++j)
            if ((v[j] = kB64.v[q[j]]) < 0) return false;
        const uint32_t x = (uint32_t)v[0] << 18 | (uint32_t)v[1] << 12 | (uint32_t)v[2] << 6 | (uint32_t)v[3];
        o[w++] = (char)(x >> 16);
        if (pad < 2) o[w++] = (char)(x >> 8);
        if (pad < 1) o[w++] = (char)x;
    }
    out.resize(w);
    return true;
}

bool b64_decode(const std::string &in, std::string &out) { return b64_decode_range(in.data(), in.size(), out); }

void json_bytes(std::string &s, const uint8_t *p, size_t n, bool null_if_empty) {
    if (!n && null_if_empty) {
        s += "null";
        return;
    }
    s.push_back('"');
    b64_encode(s, p, n);
    s.push_back('"');
}

// ValRequest / EchoRequest{ValRequest} (rbc/request.go:9-17)
std::string json_val(const uint8_t *root, size_t rl, const uint8_t *branch, size_t bl, const uint8_t *block,
                     size_t kl) {
    std::string s;
    s.reserve(64 + 4 * ((rl + 2) / 3) + 4 * ((bl + 2) / 3) + 4 * ((kl + 2) / 3));
    s = "{\"RootHash\":";
    json_bytes(s, root, rl, true);
    s += ",\"Branch\":";
    json_bytes(s, branch, bl, true);
    s += ",\"Block\":";
    if (kl) {
        s.push_back('[');
        json_bytes(s, block, kl, false);
        s.push_back(']');
    } else {
        s += "null";
    }
    s.push_back('}');
    return s;
}

// ReadyRequest (rbc/request.go:19-21)
std::string json_ready(const uint8_t *root, size_t rl) {
    std::string s = "{\"RootHash\":";
    json_bytes(s, root, rl, true);
    s.push_back('}');
    return s;
}

// Minimal JSON reader for the request shapes: an object whose fields are
// strings, null or arrays of strings; other values are skipped.  Keys match
// case-insensitively and unknown keys are ignored, as encoding/json does.
struct JsonIn {
    const char *p, *e;
    void ws() {
        while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
    }
    bool peek(char c) {
        ws();
        return p < e && *p == c;
    }
    bool eat(char c) {
        if (!peek(c)) return false;
        ++p;
        return true;
    }
    bool lit(const char *w) {
        ws();
        const size_t n = strlen(w);
        if ((size_t)(e - p) < n || memcmp(p, w, n)) return false;
        p += n;
        return true;
    }
    bool str(std::string &out) {
        if (!eat('"')) return false;
        out.clear();
        // plain run up to the closing quote (no escapes / control bytes): one copy
        const char *q = p;
        while (q < e && *q != '"' && *q != '\\' && (unsigned char)*q >= 0x20) ++q;
        out.assign(p, q);
        p = q;
        while (p < e && *p != '"') {
            char c = *p++;
            if ((unsigned char)c < 0x20) return false;
            if (c != '\\') {
                out.push_back(c);
                continue;
            }
            if (p >= e) return false;
            c = *p++;
            switch (c) {
                case '"': case '\\': case '/': out.push_back(c); break;
                case 'b': out.push_back('\b'); break;
                case 'f': out.push_back('\f'); break;
                case 'n': out.push_back('\n'); break;
                case 'r': out.push_back('\r'); break;
                case 't': out.push_back('\t'); break;
                case 'u': {
                    if (e - p < 4) return false;
                    unsigned v = 0;
                    for (int i = 0; i < 4; ++i) {
                        const char h = *p++;
                        v <<= 4;
                        if (h >= '0' && h <= '9') v |= h - '0';
                        else if (h >= 'a' && h <= 'f') v |= h - 'a' + 10;
                        else if (h >= 'A' && h <= 'F') v |= h - 'A' + 10;
                        else return false;
                    }
                    // only ASCII can be base64: anything else fails decoding later
                    out.push_back(v < 0x80 ? (char)v : '\x01');
                    break;
                }
                default: return false;
            }
        }
        if (p >= e) return false;
        ++p;
        return true;
    }
    bool skip_value(int depth = 0) {
        ws();
        if (p >= e || depth > 64) return false;
        std::string tmp;
        switch (*p) {
            case '"': return str(tmp);
            case 'n': return lit("null");
            case 't': return lit("true");
            case 'f': return lit("false");
            case '[':
                ++p;
                if (eat(']')) return true;
                do {
                    if (!skip_value(depth + 1)) return false;
                } while (eat(','));
                return eat(']');
            case '{':
                ++p;
                if (eat('}')) return true;
                do {
                    if (!str(tmp) || !eat(':') || !skip_value(depth + 1)) return false;
                } while (eat(','));
                return eat('}');
            default: {
                const char *s = p;
                while (p < e && (strchr("+-.eE", *p) || (*p >= '0' && *p <= '9'))) ++p;
                return p > s;
            }
        }
    }
    // a []byte field: base64 string or null
    bool bytes(std::string &out) {
        if (lit("null")) {
            out.clear();
            return true;
        }
        // common case, a string without escapes: decode in place
        if (peek('"')) {
            const char *q = p + 1;
            while (q < e && *q != '"' && *q != '\\' && (unsigned char)*q >= 0x20) ++q;
            if (q < e && *q == '"') {
                const char *b = p + 1;
                p = q + 1;
                return b64_decode_range(b, (size_t)(q - b), out);
            }
        }
        std::string s;
        return str(s) && b64_decode(s, out);
    }
};

bool key_is(const std::string &k, const char *want) {
    if (k.size() != strlen(want)) return false;
    for (size_t i = 0; i < k.size(); ++i) {
        char a = k[i], b = want[i];
        if (a >= 'A' && a <= 'Z') a += 32;
        if (b >= 'A' && b <= 'Z') b += 32;
        if (a != b) return false;
    }
    return true;
}

struct Request {
    std::string root, branch;
    std::vector<std::string> block;
};

// json.Unmarshal into ValRequest / EchoRequest / ReadyRequest (the caller
// checks the fields its type has).  A [][]byte field takes an array of
// base64 strings / nulls, or null.
bool json_parse(const uint8_t *in, size_t len, Request &r) {
    JsonIn j{(const char *)in, (const char *)in + len};
    if (!j.eat('{')) return false;
    if (!j.eat('}')) {
        do {
            std::string key;
            if (!j.str(key) || !j.eat(':')) return false;
            if (key_is(key, "RootHash")) {
                if (!j.bytes(r.root)) return false;
            } else if (key_is(key, "Branch")) {
                if (!j.bytes(r.branch)) return false;
            } else if (key_is(key, "Block")) {
                r.block.clear();
                if (j.lit("null")) continue;
                if (!j.eat('[')) return false;
                if (j.eat(']')) continue;
                do {
                    std::string b;
                    if (!j.bytes(b)) return false;
                    r.block.push_back(std::move(b));
                } while (j.eat(','));
                if (!j.eat(']')) return false;
            } else if (!j.skip_value()) {
                return false;
            }
        } while (j.eat(','));
        if (!j.eat('}')) return false;
    }
    j.ws();
    return j.p == j.e;
}

size_t emit(const std::string &s, uint8_t *out, size_t cap) {
    if (out && s.size() <= cap) memcpy(out, s.data(), s.size());
    return s.size();
}

// ---------------------------------------------------------------------------
// instance state
// ---------------------------------------------------------------------------
enum OpKind { OP_SHARD, OP_VAL, OP_ECHO, OP_INTERP };

// One GPU submission; heap-held so the buffers the batcher reads stay put.
struct Op {
    OpKind kind;
    uint64_t ticket = 0;
    int submit_rc = RBC_OK;
    int sender = -1;
    int ok = 0;
    Request req;  // VAL / ECHO
    // OP_SHARD
    std::string value;
    std::vector<uint8_t> shards, branches;
    size_t S = 0;
    uint8_t root[32] = {};
    // OP_INTERP
    std::string iroot;
    std::vector<const uint8_t *> ptrs;
    std::vector<size_t> lens;
    std::vector<uint8_t> out;
    size_t out_len = 0;
};

struct RootState {
    std::vector<std::string> echo;  // valid ECHO shard per sender ("" = none)
    int echoes = 0;
    std::vector<char> ready;
    int readies = 0;
    bool interp_inflight = false, interp_failed = false, have_value = false;
    std::vector<uint8_t> value;
};

struct Out {
    int to;
    std::string bytes;
};

}  // namespace

// The broadcast value is framed as [u64 little-endian length][value] before
// Split, so delivery returns exactly the proposed bytes: interpolate alone
// yields k*S bytes with the zero pad (rbc/rbc.go:86-90 carries no length).
constexpr size_t kFrame = 8;

struct rbc_node {
    rbc_batcher *b = nullptr;
    int n = 0, f = 0, k = 0, depth = 0, self = 0, proposer = 0;
    bool proposed = false, val_seen = false, ready_sent = false, delivered = false, value_ok = false;
    std::vector<char> echo_from, ready_from;  // first message per sender only
    std::map<std::string, RootState> roots;
    std::string delivered_root;
    std::vector<uint8_t> value;
    std::deque<std::unique_ptr<Op>> ops;
    std::deque<Out> outq;
    int rejected = 0;

    RootState &state(const std::string &root) {
        RootState &s = roots[root];
        if (s.echo.empty()) {
            s.echo.assign(n, std::string());
            s.ready.assign(n, 0);
        }
        return s;
    }

    void send(int to, int type, const std::string &payload) {
        outq.push_back(Out{to, pb_rbc(type, (const uint8_t *)payload.data(), payload.size())});
    }

    // Go-form branch of leaf j from the device form [n][depth][32]: the empty
    // level-0 sibling of an odd last leaf is omitted (rbc_validate_message)
    std::string flat_branch(const std::vector<uint8_t> &br, int j) const {
        std::string s;
        for (int l = 0; l < depth; ++l) {
            if (l == 0 && (j ^ 1) >= n) continue;
            s.append((const char *)br.data() + ((size_t)j * depth + l) * 32, 32);
        }
        return s;
    }

    void submit_validate(std::unique_ptr<Op> op, int index) {
        const Request &r = op->req;
        const std::string &blk = r.block[0];
        op->submit_rc = rbc_batcher_validate(b, (const uint8_t *)r.root.data(), (const uint8_t *)r.branch.data(),
                                             r.branch.size(), (const uint8_t *)blk.data(), blk.size(),
                                             (uint32_t)index, &op->ok, &op->ticket);
        ops.push_back(std::move(op));
    }

    void submit_interp(const std::string &root, RootState &s) {
        auto op = std::make_unique<Op>();
        op->kind = OP_INTERP;
        op->iroot = root;
        // snapshot by reference: an ECHO slot is written once and never again,
        // and a root's state is never erased, so the shards the launch reads
        // stay in place while later ECHOs fill other slots
        op->ptrs.resize(n);
        op->lens.resize(n);
        size_t S = 1;
        for (int j = 0; j < n; ++j) {
            op->ptrs[j] = (const uint8_t *)s.echo[j].data();
            op->lens[j] = s.echo[j].size();
            if (op->lens[j]) S = op->lens[j];
        }
        op->out.resize((size_t)k * S);
        s.interp_inflight = true;
        op->submit_rc = rbc_batcher_interpolate(b, (const uint8_t *)op->iroot.data(), op->ptrs.data(),
                                                op->lens.data(), op->out.data(), op->out.size(), &op->out_len,
                                                nullptr, &op->ticket);
        ops.push_back(std::move(op));
    }

    // our VAL (own or received) proved our shard: ECHO it to every other node,
    // the proposer included, and count our own ECHO here.  HBBFT's "multicast
    // ECHO" (Miller et al. 2016, Algorithm RBC), not docs/RBC-EN.md:34 ("except
    // the sender and itself"): without ECHOs the proposer could never decode
    // (RBC-EN.md:42) and would not deliver its own value
    // (the shard moves into our ECHO slot: the bytes the VAL's validate read,
    // at the same address -- a batcher that keeps validated rows on the device
    // finds them again for the interpolate)
    void on_val(Request &r) {
        send(-1, RBC_MSG_ECHO,
             json_val((const uint8_t *)r.root.data(), r.root.size(), (const uint8_t *)r.branch.data(),
                      r.branch.size(), (const uint8_t *)r.block[0].data(), r.block[0].size()));
        on_echo(self, r.root, std::move(r.block[0]));
    }

    void on_echo(int from, const std::string &root, std::string &&shard) {
        RootState &s = state(root);
        if (s.echo[from].empty()) {
            s.echo[from] = std::move(shard);
            s.echoes++;
        }
        advance(root);
    }

    void on_ready(int from, const std::string &root) {
        RootState &s = state(root);
        if (!s.ready[from]) {
            s.ready[from] = 1;
            s.readies++;
        }
        advance(root);
    }

    void send_ready(const std::string &root) {
        if (ready_sent) return;
        ready_sent = true;
        send(-1, RBC_MSG_READY, json_ready((const uint8_t *)root.data(), root.size()));
        on_ready(self, root);
    }

    // HBBFT thresholds for one root (docs/RBC-EN.md)
    void advance(const std::string &root) {
        RootState &s = state(root);
        // N-f ECHOs: interpolate, READY on a root match.  2f+1 READYs with
        // N-2f ECHOs: interpolate to deliver, even if we never saw N-f ECHOs.
        if (!s.have_value && !s.interp_inflight && !s.interp_failed &&
            ((s.echoes >= n - f && !ready_sent) || (s.readies >= 2 * f + 1 && s.echoes >= n - 2 * f)))
            submit_interp(root, s);
        if (s.readies >= f + 1) send_ready(root);  // amplification
        if (!delivered && s.have_value && s.readies >= 2 * f + 1 && s.echoes >= n - 2 * f) {
            delivered = true;
            delivered_root = root;
            // unframe: [u64 LE length][value][Split zero pad].  Every honest
            // node decodes the same k*S bytes, so a bad length (a Byzantine
            // proposer's) is seen identically everywhere: delivered, unusable.
            uint64_t L = 0;
            if (s.value.size() >= kFrame) {
                for (int b = 0; b < 8; ++b) L |= (uint64_t)s.value[b] << (8 * b);
                value_ok = L <= s.value.size() - kFrame;
            }
            if (value_ok) value.assign(s.value.begin() + kFrame, s.value.begin() + kFrame + (size_t)L);
        }
    }

    void complete(Op &op) {
        int st = op.submit_rc;
        if (!st && op.ticket) st = rbc_batcher_wait(b, op.ticket);
        switch (op.kind) {
            case OP_SHARD: {
                if (st) {
                    rejected++;
                    break;
                }
                const std::string root((const char *)op.root, 32);
                Request own;
                for (int j = 0; j < n; ++j) {
                    Request r;
                    r.root = root;
                    r.branch = flat_branch(op.branches, j);
                    r.block.emplace_back((const char *)op.shards.data() + (size_t)j * op.S, op.S);
                    if (j == self)
                        own = std::move(r);
                    else
                        send(j, RBC_MSG_VAL,
                             json_val((const uint8_t *)r.root.data(), 32, (const uint8_t *)r.branch.data(),
                                      r.branch.size(), (const uint8_t *)r.block[0].data(), op.S));
                }
                on_val(own);
                break;
            }
            case OP_VAL:
                if (st || !op.ok) {
                    rejected++;
                    break;
                }
                on_val(op.req);
                break;
            case OP_ECHO:
                if (st || !op.ok) {  // the sender's one ECHO slot stays used
                    rejected++;
                    break;
                }
                on_echo(op.sender, op.req.root, std::move(op.req.block[0]));
                break;
            case OP_INTERP: {
                RootState &s = state(op.iroot);
                s.interp_inflight = false;
                if (st) {  // not a codeword under this root: never READY for it
                    s.interp_failed = true;
                    break;
                }
                s.have_value = true;
                s.value.assign(op.out.begin(), op.out.begin() + op.out_len);
                send_ready(op.iroot);
                advance(op.iroot);
                break;
            }
        }
    }
};

extern "C" {

size_t rbc_pb_encode_rbc(int type, const uint8_t *payload, size_t payload_len, uint8_t *out, size_t cap) {
    return emit(pb_rbc(type, payload, payload ? payload_len : 0), out, cap);
}

int rbc_pb_decode_rbc(const uint8_t *msg, size_t len, int *type, const uint8_t **payload, size_t *payload_len) {
    if ((!msg && len) || !type || !payload || !payload_len) return RBC_ERR_INVALID_ARG;
    return pb_parse(msg, len, type, payload, payload_len);
}

size_t rbc_json_encode_val(const uint8_t *root, size_t root_len, const uint8_t *branch, size_t branch_len,
                           const uint8_t *block, size_t block_len, uint8_t *out, size_t cap) {
    return emit(json_val(root, root ? root_len : 0, branch, branch ? branch_len : 0, block, block ? block_len : 0),
                out, cap);
}

size_t rbc_json_encode_ready(const uint8_t *root, size_t root_len, uint8_t *out, size_t cap) {
    return emit(json_ready(root, root ? root_len : 0), out, cap);
}

int rbc_json_decode_val(const uint8_t *json, size_t len, uint8_t *root_out, uint8_t *branch_out, size_t branch_cap,
                        size_t *branch_len, uint8_t *block_out, size_t block_cap, size_t *block_len) {
    if ((!json && len) || !root_out || !branch_len || !block_len) return RBC_ERR_INVALID_ARG;
    Request r;
    if (!json_parse(json, len, r) || r.root.size() != 32 || r.block.size() != 1) return RBC_ERR_PROTOCOL;
    *branch_len = r.branch.size();
    *block_len = r.block[0].size();
    if (r.branch.size() > branch_cap || r.block[0].size() > block_cap) return RBC_ERR_INVALID_ARG;
    memcpy(root_out, r.root.data(), 32);
    if (branch_out) memcpy(branch_out, r.branch.data(), r.branch.size());
    if (block_out) memcpy(block_out, r.block[0].data(), r.block[0].size());
    return RBC_OK;
}

int rbc_json_decode_ready(const uint8_t *json, size_t len, uint8_t *root_out) {
    if ((!json && len) || !root_out) return RBC_ERR_INVALID_ARG;
    Request r;
    if (!json_parse(json, len, r) || r.root.size() != 32) return RBC_ERR_PROTOCOL;
    memcpy(root_out, r.root.data(), 32);
    return RBC_OK;
}

int rbc_node_create(rbc_batcher *batcher, int n, int f, int self, int proposer, rbc_node **out) {
    // n >= 3f + 1: the HBBFT thresholds (N-f ECHO, f+1 / 2f+1 READY) need it
    // for quorum intersection (the raw data-path context stays permissive)
    if (!batcher || !out || n < 1 || f < 0 || n < 3 * f + 1 || self < 0 || self >= n || proposer < 0 ||
        proposer >= n)
        return RBC_ERR_INVALID_ARG;
    rbc_node *node = new rbc_node();
    node->b = batcher;
    node->n = n;
    node->f = f;
    node->k = n - 2 * f;
    int d = 0;
    while ((1 << d) < n) ++d;
    node->depth = d;
    node->self = self;
    node->proposer = proposer;
    node->echo_from.assign(n, 0);
    node->ready_from.assign(n, 0);
    *out = node;
    return RBC_OK;
}

void rbc_node_destroy(rbc_node *node) {
    if (!node) return;
    for (auto &op : node->ops)  // the batcher may still read these buffers
        if (!op->submit_rc && op->ticket) rbc_batcher_wait(node->b, op->ticket);
    delete node;
}

int rbc_node_propose(rbc_node *node, const uint8_t *value, size_t len) {
    if (!node || (!value && len)) return RBC_ERR_INVALID_ARG;
    if (node->self != node->proposer || node->proposed) return RBC_ERR_PROTOCOL;
    node->proposed = true;  // an empty value is a valid (framed, 8-byte) proposal
    auto op = std::make_unique<Op>();
    op->kind = OP_SHARD;
    op->value.resize(kFrame);
    for (size_t b = 0; b < kFrame; ++b) op->value[b] = (char)((uint64_t)len >> (8 * b));
    op->value.append((const char *)value, len);
    len = op->value.size();
    op->S = (len + node->k - 1) / node->k;
    op->shards.resize((size_t)node->n * op->S);
    op->branches.resize((size_t)node->n * (node->depth ? node->depth : 1) * 32);
    op->submit_rc = rbc_batcher_shard(node->b, (const uint8_t *)op->value.data(), len, op->shards.data(),
                                      op->shards.size(), &op->S, op->root, op->branches.data(), &op->ticket);
    const int rc = op->submit_rc;
    node->ops.push_back(std::move(op));
    return rc;
}

int rbc_node_handle_message(rbc_node *node, int sender, const uint8_t *msg, size_t len) {
    if (!node || sender < 0 || sender >= node->n || (!msg && len)) return RBC_ERR_INVALID_ARG;
    int type;
    const uint8_t *pl;
    size_t pll;
    Request r;
    if (pb_parse(msg, len, &type, &pl, &pll) != RBC_OK || !json_parse(pl, pll, r) || r.root.size() != 32) {
        node->rejected++;
        return RBC_ERR_PROTOCOL;
    }
    if (type == RBC_MSG_READY) {  // handleReadyRequest: one READY per sender
        if (node->ready_from[sender] || sender == node->self) {
            node->rejected++;
            return RBC_ERR_PROTOCOL;
        }
        node->ready_from[sender] = 1;
        node->on_ready(sender, r.root);
        return RBC_OK;
    }
    const bool val = type == RBC_MSG_VAL;
    // handleValueRequest: only the proposer's first VAL (it carries our
    // shard); handleEchoRequest: the first ECHO per sender (its shard)
    const bool dup = val ? (sender != node->proposer || node->val_seen)
                         : (node->echo_from[sender] || sender == node->self);
    if (dup || r.block.size() != 1 || r.block[0].empty()) {
        node->rejected++;
        return RBC_ERR_PROTOCOL;
    }
    auto op = std::make_unique<Op>();
    op->sender = sender;
    op->req = std::move(r);
    if (val) {
        node->val_seen = true;
        op->kind = OP_VAL;
        node->submit_validate(std::move(op), node->self);
    } else {
        node->echo_from[sender] = 1;
        op->kind = OP_ECHO;
        node->submit_validate(std::move(op), sender);
    }
    return RBC_OK;
}

int rbc_node_progress(rbc_node *node, int wait, int *pending_out) {
    if (!node) return RBC_ERR_INVALID_ARG;
    while (!node->ops.empty()) {
        Op &op = *node->ops.front();
        if (!wait && !op.submit_rc && op.ticket) {
            int done = 0;
            rbc_batcher_poll(node->b, op.ticket, &done);
            if (!done) break;
        }
        std::unique_ptr<Op> hold = std::move(node->ops.front());
        node->ops.pop_front();
        node->complete(*hold);  // may queue new submissions behind
    }
    if (pending_out) *pending_out = (int)node->ops.size();
    return RBC_OK;
}

int rbc_node_next_message(rbc_node *node, int *to, uint8_t *buf, size_t cap, size_t *len) {
    if (!node || !to || !len) return RBC_ERR_INVALID_ARG;
    if (node->outq.empty()) {
        *len = 0;
        *to = -1;
        return RBC_OK;
    }
    const Out &o = node->outq.front();
    *len = o.bytes.size();
    *to = o.to;
    if (!buf || o.bytes.size() > cap) return RBC_ERR_INVALID_ARG;
    memcpy(buf, o.bytes.data(), o.bytes.size());
    node->outq.pop_front();
    return RBC_OK;
}

int rbc_node_value(rbc_node *node, uint8_t *buf, size_t cap, size_t *len, int *delivered) {
    if (!node || !len || !delivered) return RBC_ERR_INVALID_ARG;
    *delivered = node->delivered;
    *len = node->delivered ? node->value.size() : 0;
    if (node->delivered && !node->value_ok) return RBC_ERR_PROTOCOL;  // agreed on, but badly framed
    if (!node->delivered || (!buf && cap == 0)) return RBC_OK;  // NULL buffer: size query
    if (!buf || node->value.size() > cap) return RBC_ERR_INVALID_ARG;
    memcpy(buf, node->value.data(), node->value.size());
    return RBC_OK;
}

int rbc_node_stats(rbc_node *node, int *echoes, int *readies, int *ready_sent, int *rejected) {
    if (!node) return RBC_ERR_INVALID_ARG;
    const RootState *lead = nullptr;
    if (node->delivered) {
        lead = &node->roots[node->delivered_root];
    } else {
        for (auto &kv : node->roots)
            if (!lead || kv.second.echoes + kv.second.readies > lead->echoes + lead->readies) lead = &kv.second;
    }
    if (echoes) *echoes = lead ? lead->echoes : 0;
    if (readies) *readies = lead ? lead->readies : 0;
    if (ready_sent) *ready_sent = node->ready_sent;
    if (rejected) *rejected = node->rejected;
    return RBC_OK;
}

}  // extern "C"
