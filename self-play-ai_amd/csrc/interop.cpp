// interop.cpp — safetensors checkpoints with tch VarStore naming.
//
// The reference saves and loads its nets with VarStore::save/load
// (learner.rs:192, learner_concurrent.rs:155-156, main.rs:61).  tch 0.13 keys
// every variable by its path name on the root path; a name already present
// gets the suffix "__<number of variables in the store>" (nn::Path::add).
// Construction order (model/mod.rs:167-184, model/connect_four.rs:54-72,
// model/tictactoe.rs:54-72, model/chess.rs:48-70): stem, residual blocks,
// policy head, value head.  The variable-creation order INSIDE each tch module
// decides every "__N" suffix; it is the one table below (kModuleOrder).  tch is
// not vendored, so that table is restated from tch 0.13's nn/conv.rs,
// nn/linear.rs and nn/batch_norm.rs as recalled: PARITY UNPINNED -- no
// tch-written checkpoint exists here to check it against.  The file format
// itself is checked against the safetensors package in the tests, and the
// loader names the first tensor it cannot match (name, shape or dtype).
// File format: u64 little-endian header length, a JSON header
// {"name": {"dtype": "F32", "shape": [...], "data_offsets": [begin, end]}, ...}
// and the raw little-endian tensor bytes.
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "spai_internal.h"

namespace spai {
namespace {

struct TensorSpec {
    std::string name;
    std::vector<int64_t> shape;
    size_t offset;   // into the flat parameter vector (floats)
    size_t count;
};

// Variable-creation order inside one tch module (the single place to correct if
// a real tch checkpoint disagrees).  The flat parameter vector of spai_net_create
// always stores weight before bias; only the names follow this order.
struct ModuleOrder {
    bool conv_bias_first;     // nn::conv2d: `bias` var created before `weight`
    bool linear_bias_first;   // nn::linear: `bias` var created before `weight`
    // nn::batch_norm2d: weight, bias, running_mean, running_var (fixed)
};
constexpr ModuleOrder kModuleOrder{true, true};

// A net's variables in flat order, with tch names (VarStore: a repeated name gets
// "__<variables created so far>", nn::Path::add) and shapes.
struct SpecBuilder {
    std::vector<TensorSpec> out;
    std::map<std::string, int> seen;
    size_t created = 0;   // variables created so far (tch's suffix counter)
    size_t off = 0;       // flat offset
    std::string name(const std::string &base) {
        std::string n = seen.count(base) ? base + "__" + std::to_string(created) : base;
        seen[base] = 1;
        ++created;
        return n;
    }
    void push(const std::string &nm, std::vector<int64_t> shape) {
        size_t n = 1;
        for (int64_t d : shape) n *= (size_t)d;
        out.push_back({nm, shape, off, n});
        off += n;
    }
    void weight_bias(bool bias_first, std::vector<int64_t> wshape, int64_t nb) {
        std::string w, b;
        if (bias_first) {
            b = name("bias");
            w = name("weight");
        } else {
            w = name("weight");
            b = name("bias");
        }
        push(w, wshape);   // flat order: weight, bias
        push(b, {nb});
    }
    void conv(int64_t ci, int64_t co, int64_t k) { weight_bias(kModuleOrder.conv_bias_first, {co, ci, k, k}, co); }
    void bn(int64_t c) {
        for (const char *v : {"weight", "bias", "running_mean", "running_var"}) push(name(v), {c});
    }
    void conv_bn(int64_t ci, int64_t co) {
        conv(ci, co, 3);
        bn(co);
    }
    void linear(int64_t in, int64_t outf) { weight_bias(kModuleOrder.linear_bias_first, {outf, in}, outf); }
};

// Connect4 (model/connect_four.rs:50-72) and TicTacToe (model/tictactoe.rs:50-72):
// torso (model/mod.rs:167-184), policy head conv 32 + linear, value head conv 3 + linear
// chess (model/chess.rs:48-70): torso, policy head 1x1 convs (no BN), value head 1x1 conv + 2 linears
std::vector<TensorSpec> net_specs(int game, int blocks, int hidden) {
    SpecBuilder b;
    if (game == SPAI_GAME_CHESS) {
        b.conv_bn(19, hidden);
        for (int i = 0; i < 2 * blocks; ++i) b.conv_bn(hidden, hidden);
        b.conv(hidden, 256, 1);
        b.conv(256, 73, 1);
        b.conv(hidden, 1, 1);
        b.linear(64, 256);
        b.linear(256, 1);
        return b.out;
    }
    const int64_t cells = game == SPAI_GAME_TICTACTOE ? 9 : 42, actions = game == SPAI_GAME_TICTACTOE ? 9 : 7;
    b.conv_bn(3, hidden);
    for (int i = 0; i < 2 * blocks; ++i) b.conv_bn(hidden, hidden);
    b.conv_bn(hidden, 32);
    b.linear(32 * cells, actions);
    b.conv_bn(hidden, 3);
    b.linear(3 * cells, 1);
    return b.out;
}

size_t specs_total(const std::vector<TensorSpec> &v) { return v.empty() ? 0 : v.back().offset + v.back().count; }

// ---- a minimal JSON reader for the safetensors header (objects, strings, integer arrays)
struct Json {
    const char *p, *end;
    bool ok = true;
    void ws() {
        while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
    }
    bool eat(char c) {
        ws();
        if (p < end && *p == c) {
            ++p;
            return true;
        }
        return false;
    }
    std::string str() {
        ws();
        std::string s;
        if (p >= end || *p != '"') {
            ok = false;
            return s;
        }
        ++p;
        while (p < end && *p != '"') {
            if (*p == '\\' && p + 1 < end) ++p;
            s += *p++;
        }
        if (p < end) ++p;
        else ok = false;
        return s;
    }
    int64_t integer() {
        ws();
        int64_t v = 0;
        bool neg = false, any = false;
        if (p < end && *p == '-') {
            neg = true;
            ++p;
        }
        while (p < end && *p >= '0' && *p <= '9') {
            v = v * 10 + (*p++ - '0');
            any = true;
        }
        if (!any) ok = false;
        return neg ? -v : v;
    }
    std::vector<int64_t> int_array() {
        std::vector<int64_t> v;
        if (!eat('[')) {
            ok = false;
            return v;
        }
        if (eat(']')) return v;
        do v.push_back(integer());
        while (ok && eat(','));
        if (!eat(']')) ok = false;
        return v;
    }
    void skip_value() {   // strings, numbers, nested objects/arrays (for __metadata__)
        ws();
        if (p >= end) {
            ok = false;
            return;
        }
        if (*p == '"') {
            str();
        } else if (*p == '{' || *p == '[') {
            const char open = *p, close = open == '{' ? '}' : ']';
            int depth = 0;
            do {
                if (*p == '"') {
                    str();
                    continue;
                }
                if (*p == open) ++depth;
                if (*p == close) --depth;
                ++p;
            } while (p < end && depth > 0);
        } else {
            while (p < end && *p != ',' && *p != '}' && *p != ']') ++p;
        }
    }
};

struct Entry {
    std::string dtype;
    std::vector<int64_t> shape;
    int64_t begin = -1, end = -1;
};

}  // namespace

int params_save_safetensors(int game, int blocks, int hidden, const float *params, size_t n, const char *path) {
    SPAI_CHECK(game >= SPAI_GAME_TICTACTOE && game <= SPAI_GAME_CHESS, SPAI_ERR_INVALID, "bad game %d", game);
    SPAI_CHECK(blocks >= 0 && hidden > 0, SPAI_ERR_INVALID, "bad net shape");
    const std::vector<TensorSpec> specs = net_specs(game, blocks, hidden);
    SPAI_CHECK(n == specs_total(specs), SPAI_ERR_INVALID, "expected %zu params, got %zu", specs_total(specs), n);
    std::string h = "{\"__metadata__\":{\"format\":\"pt\"}";
    size_t byte = 0;
    for (const TensorSpec &t : specs) {
        h += ",\"" + t.name + "\":{\"dtype\":\"F32\",\"shape\":[";
        for (size_t i = 0; i < t.shape.size(); ++i) h += (i ? "," : "") + std::to_string(t.shape[i]);
        h += "],\"data_offsets\":[" + std::to_string(byte) + "," + std::to_string(byte + 4 * t.count) + "]}";
        byte += 4 * t.count;
    }
    h += "}";
    while ((8 + h.size()) % 8) h += ' ';   // align the data block to 8 bytes (spec allows trailing spaces)
    FILE *f = std::fopen(path, "wb");
    SPAI_CHECK(f, SPAI_ERR_INVALID, "cannot open %s for writing", path);
    const uint64_t hl = h.size();
    uint8_t le[8];
    for (int i = 0; i < 8; ++i) le[i] = (uint8_t)(hl >> (8 * i));
    bool ok = std::fwrite(le, 1, 8, f) == 8 && std::fwrite(h.data(), 1, h.size(), f) == h.size();
    for (const TensorSpec &t : specs)   // construction order = flat order: one contiguous write
        ok = ok && std::fwrite(params + t.offset, 4, t.count, f) == t.count;
    ok = (std::fclose(f) == 0) && ok;
    SPAI_CHECK(ok, SPAI_ERR_INVALID, "write to %s failed", path);
    return SPAI_OK;
}

int params_load_safetensors(int game, int blocks, int hidden, const char *path, float *params, size_t n) {
    SPAI_CHECK(game >= SPAI_GAME_TICTACTOE && game <= SPAI_GAME_CHESS, SPAI_ERR_INVALID, "bad game %d", game);
    SPAI_CHECK(blocks >= 0 && hidden > 0, SPAI_ERR_INVALID, "bad net shape");
    const std::vector<TensorSpec> specs = net_specs(game, blocks, hidden);
    SPAI_CHECK(n == specs_total(specs), SPAI_ERR_INVALID, "expected %zu params, got %zu", specs_total(specs), n);
    FILE *f = std::fopen(path, "rb");
    SPAI_CHECK(f, SPAI_ERR_INVALID, "cannot open %s", path);
    std::vector<uint8_t> buf;
    {
        uint8_t tmp[1 << 16];
        size_t r;
        while ((r = std::fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + r);
        std::fclose(f);
    }
    SPAI_CHECK(buf.size() >= 8, SPAI_ERR_INVALID, "%s: not a safetensors file", path);
    uint64_t hl = 0;
    for (int i = 0; i < 8; ++i) hl |= (uint64_t)buf[i] << (8 * i);
    SPAI_CHECK(hl <= buf.size() - 8, SPAI_ERR_INVALID, "%s: header length %llu past the end", path,
               (unsigned long long)hl);
    const uint8_t *data = buf.data() + 8 + hl;
    const size_t data_len = buf.size() - 8 - hl;
    Json js{(const char *)buf.data() + 8, (const char *)buf.data() + 8 + hl};
    std::map<std::string, Entry> entries;
    SPAI_CHECK(js.eat('{'), SPAI_ERR_INVALID, "%s: bad header", path);
    if (!js.eat('}')) {
        do {
            const std::string key = js.str();
            SPAI_CHECK(js.ok && js.eat(':'), SPAI_ERR_INVALID, "%s: bad header near '%s'", path, key.c_str());
            if (key == "__metadata__") {
                js.skip_value();
                continue;
            }
            Entry e;
            SPAI_CHECK(js.eat('{'), SPAI_ERR_INVALID, "%s: bad entry '%s'", path, key.c_str());
            do {
                const std::string field = js.str();
                SPAI_CHECK(js.ok && js.eat(':'), SPAI_ERR_INVALID, "%s: bad entry '%s'", path, key.c_str());
                if (field == "dtype") e.dtype = js.str();
                else if (field == "shape") e.shape = js.int_array();
                else if (field == "data_offsets") {
                    const std::vector<int64_t> o = js.int_array();
                    if (o.size() == 2) {
                        e.begin = o[0];
                        e.end = o[1];
                    }
                } else js.skip_value();
            } while (js.ok && js.eat(','));
            SPAI_CHECK(js.ok && js.eat('}'), SPAI_ERR_INVALID, "%s: bad entry '%s'", path, key.c_str());
            entries[key] = e;
        } while (js.ok && js.eat(','));
        SPAI_CHECK(js.ok && js.eat('}'), SPAI_ERR_INVALID, "%s: bad header", path);
    }
    auto shape_str = [](const std::vector<int64_t> &v) {
        std::string r = "[";
        for (size_t i = 0; i < v.size(); ++i) r += (i ? "," : "") + std::to_string(v[i]);
        return r + "]";
    };
    for (const TensorSpec &t : specs) {
        auto it = entries.find(t.name);
        if (it == entries.end()) {   // name the first mismatch, with a same-shape candidate if any
            std::string cand;
            for (const auto &kv : entries)
                if (kv.second.shape == t.shape && !cand.size()) cand = kv.first;
            SPAI_CHECK(false, SPAI_ERR_INVALID,
                       "%s: missing tensor '%s' %s (tch naming is restated, parity unpinned; the file has %zu "
                       "tensors%s%s%s)", path, t.name.c_str(), shape_str(t.shape).c_str(), entries.size(),
                       cand.size() ? ", same shape: '" : "", cand.c_str(), cand.size() ? "'" : "");
        }
        const Entry &e = it->second;
        SPAI_CHECK(e.dtype == "F32", SPAI_ERR_UNSUPPORTED, "%s: tensor '%s' is %s, expected F32", path,
                   t.name.c_str(), e.dtype.c_str());
        SPAI_CHECK(e.shape == t.shape, SPAI_ERR_INVALID, "%s: tensor '%s' has shape %s, expected %s", path,
                   t.name.c_str(), shape_str(e.shape).c_str(), shape_str(t.shape).c_str());
        SPAI_CHECK(e.begin >= 0 && e.end - e.begin == (int64_t)(4 * t.count) && (size_t)e.end <= data_len,
                   SPAI_ERR_INVALID, "%s: tensor '%s' has bad data offsets", path, t.name.c_str());
        memcpy(params + t.offset, data + e.begin, 4 * t.count);   // little-endian F32 on this host
    }
    return SPAI_OK;
}

}  // namespace spai
