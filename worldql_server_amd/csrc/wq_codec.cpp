// wq_codec.cpp — batch FlatBuffer decode of WorldQL Message frames and world-name sanitizing
// (include/wq_codec.h). Host C++ only.
//
// Decode = the reference's Message::deserialize (structures/message.rs:136-142):
//   1. root_as_message (WorldQLFB_generated.rs:1192-1194): the FlatBuffers 2.0.0 Rust verifier over
//      the Message table (:986-1004, Record :515-527, Entity :734-746) — every offset aligned
//      (relative to the frame start) and in bounds, vtables even-sized and in bounds, strings valid
//      UTF-8 with a NUL after them, vectors in bounds;
//   2. MessageT -> Message (message.rs:60-114): world_name and sender_uuid required, every Record
//      (record.rs:30-50: uuid, world_name required) and Entity (entity.rs:29-48: uuid, position,
//      world_name required) decoded, uuids parsed with uuid 0.8.2's parse_str; instruction codes
//      outside 0..12 become Unknown, replication codes outside 0..2 ExceptSelf.
// Limits the verifier also enforces but no WorldQL frame can reach are kept as well (table count
// 1,000,000, depth 64, apparent size 2^31).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "wq_codec.h"

namespace {

// ---- verifier (flatbuffers 2.0.0, src/verifier.rs) ------------------------------------------
struct Verifier {
    const uint8_t* b;
    size_t n;
    size_t apparent = 0;
    size_t tables = 0;
    int depth = 0;
    bool ok = true;

    bool fail() { return ok = false; }
    bool aligned(size_t pos, size_t a) { return (pos % a == 0) || fail(); }
    bool range(size_t pos, size_t size) {
        const size_t end = pos + size < pos ? SIZE_MAX : pos + size;  // saturating_add
        if (end > n) return fail();
        apparent += size;
        if (apparent > (size_t(1) << 31)) return fail();
        return true;
    }
    uint32_t rd32(size_t p) const { uint32_t v; memcpy(&v, b + p, 4); return v; }
    uint16_t rd16(size_t p) const { uint16_t v; memcpy(&v, b + p, 2); return v; }
    bool u32_at(size_t pos, uint32_t* v) {  // get_uoffset: aligned 4, in range
        if (!aligned(pos, 4) || !range(pos, 4)) return false;
        *v = rd32(pos);
        return true;
    }
    bool u16_at(size_t pos, uint16_t* v) {
        if (!aligned(pos, 2) || !range(pos, 2)) return false;
        *v = rd16(pos);
        return true;
    }
    // ForwardsUOffset: pos -> pos + uoffset (saturating)
    bool follow(size_t pos, size_t* out) {
        uint32_t off;
        if (!u32_at(pos, &off)) return false;
        *out = pos + off < pos ? SIZE_MAX : pos + off;
        return true;
    }
    // vector header at pos: element range [start, start + len * elem)
    bool vec_range(size_t pos, size_t elem, size_t* start, size_t* len) {
        uint32_t l;
        if (!u32_at(pos, &l)) return false;
        const size_t s = pos + 4 < pos ? SIZE_MAX : pos + 4;
        if (!aligned(s, elem)) return false;
        const size_t size = (size_t)l * elem;
        if (!range(s, size)) return false;
        *start = s;
        *len = l;
        return true;
    }
};

// Rust std::str::from_utf8 acceptance (no overlongs, no surrogates, <= U+10FFFF)
bool valid_utf8(const uint8_t* s, size_t n) {
    size_t i = 0;
    while (i < n) {
        const uint8_t c = s[i];
        if (c < 0x80) { ++i; continue; }
        size_t k;
        uint8_t lo = 0x80, hi = 0xBF;
        if (c >= 0xC2 && c <= 0xDF) k = 1;
        else if (c == 0xE0) { k = 2; lo = 0xA0; }
        else if ((c >= 0xE1 && c <= 0xEC) || c == 0xEE || c == 0xEF) k = 2;
        else if (c == 0xED) { k = 2; hi = 0x9F; }
        else if (c == 0xF0) { k = 3; lo = 0x90; }
        else if (c >= 0xF1 && c <= 0xF3) k = 3;
        else if (c == 0xF4) { k = 3; hi = 0x8F; }
        else return false;
        if (i + k >= n) return false;  // truncated sequence
        if (s[i + 1] < lo || s[i + 1] > hi) return false;
        for (size_t j = 2; j <= k; ++j)
            if (s[i + j] < 0x80 || s[i + j] > 0xBF) return false;
        i += k + 1;
    }
    return true;
}

struct Str {
    bool present = false;
    uint32_t off = 0, len = 0;
};

// &str verifier: vector of u8, UTF-8, NUL right after it (not range-checked, only read if present)
bool verify_str(Verifier& v, size_t pos, Str* s) {
    size_t start, len;
    if (!v.aligned(pos, 4) || !v.vec_range(pos, 1, &start, &len)) return false;
    const size_t end = start + len;
    if (!valid_utf8(v.b + start, len)) return v.fail();
    if (end >= v.n || v.b[end] != 0) return v.fail();
    s->present = true;
    s->off = (uint32_t)start;
    s->len = (uint32_t)len;
    return true;
}

struct Table {
    size_t pos = 0, vt = 0, vt_len = 0;
};

// visit_table: soffset to the vtable (counted against max_tables), vtable length even and in range
bool visit_table(Verifier& v, size_t pos, Table* t) {
    if (++v.tables > 1000000) return v.fail();
    uint32_t raw;
    if (!v.u32_at(pos, &raw)) return false;
    const int32_t so = (int32_t)raw;
    size_t vt;
    if (so > 0) {  // the vtable precedes the table
        if ((size_t)so > pos) return v.fail();
        vt = pos - (size_t)so;
    } else {
        const uint64_t a = (uint64_t)(-(int64_t)so);
        vt = pos + (size_t)a;
        if (vt < pos) return v.fail();
    }
    if (vt >= v.n) return v.fail();
    uint16_t vl;
    if (!v.u16_at(vt, &vl)) return false;
    if (!v.aligned(vt + vl, 2) || !v.range(vt, vl)) return false;
    if (++v.depth > 64) return v.fail();
    t->pos = pos;
    t->vt = vt;
    t->vt_len = vl;
    return true;
}

// TableVerifier::deref: field position, or 0 when absent
bool field(Verifier& v, const Table& t, size_t voff, size_t* fpos) {
    *fpos = 0;
    if (voff < t.vt_len) {
        uint16_t fo;
        if (!v.u16_at(t.vt + voff, &fo)) return false;
        if (fo > 0) *fpos = t.pos + fo;
    }
    return true;
}

bool field_str(Verifier& v, const Table& t, size_t voff, Str* s) {
    size_t fp;
    if (!field(v, t, voff, &fp)) return false;
    if (!fp) return true;
    size_t sp;
    return v.follow(fp, &sp) && verify_str(v, sp, s);
}

bool field_u8(Verifier& v, const Table& t, size_t voff, uint8_t dflt, uint8_t* out) {
    size_t fp;
    if (!field(v, t, voff, &fp)) return false;
    *out = dflt;
    if (!fp) return true;
    if (!v.range(fp, 1)) return false;
    *out = v.b[fp];
    return true;
}

bool field_vec3(Verifier& v, const Table& t, size_t voff, bool* has, double* xyz) {
    size_t fp;
    if (!field(v, t, voff, &fp)) return false;
    *has = false;
    if (!fp) return true;
    if (!v.range(fp, 24)) return false;  // Vec3d is [u8; 24]: alignment 1
    memcpy(xyz, v.b + fp, 24);
    *has = true;
    return true;
}

bool field_bytes(Verifier& v, const Table& t, size_t voff) {
    size_t fp;
    if (!field(v, t, voff, &fp)) return false;
    if (!fp) return true;
    size_t vp, s, l;
    return v.follow(fp, &vp) && v.aligned(vp, 4) && v.vec_range(vp, 1, &s, &l);
}

// ---- uuid 0.8.2 Uuid::parse_str --------------------------------------------------------------
int hexv(uint8_t c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

bool parse_uuid(const uint8_t* s, size_t len, uint8_t out[16]) {
    static const uint8_t kGroupEnd[5] = {8, 12, 16, 20, 32};  // ACC_GROUP_LENS
    if (len == 45 && memcmp(s, "urn:uuid:", 9) == 0) {
        s += 9;
        len -= 9;
    } else if (len != 32 && len != 36) {
        return false;
    }
    int digit = 0, group = 0;
    uint8_t acc = 0;
    for (size_t i = 0; i < len; ++i) {
        const uint8_t c = s[i];
        if (digit >= 32 && group != 4) return false;
        if (digit % 2 == 0) {
            const int h = hexv(c);
            if (h >= 0) {
                acc = (uint8_t)h;
            } else if (c == '-') {
                if (group > 4 || kGroupEnd[group] != digit) return false;
                ++group;
                --digit;
            } else {
                return false;
            }
        } else {
            const int h = hexv(c);
            if (h < 0) return false;
            acc = (uint8_t)(acc * 16 + h);
            out[digit / 2] = acc;
        }
        ++digit;
    }
    return digit == kGroupEnd[4];
}

// ---- Message ----------------------------------------------------------------------------------
// vtable offsets: Message (WorldQLFB_generated.rs:939-947), Record/Entity (:485-489, :704-708)
enum : size_t { M_INSTR = 4, M_PARAM = 6, M_SENDER = 8, M_WORLD = 10, M_REPL = 12, M_RECORDS = 14,
                M_ENTITIES = 16, M_POS = 18, M_FLEX = 20 };
enum : size_t { R_UUID = 4, R_POS = 6, R_WORLD = 8, R_DATA = 10, R_FLEX = 12 };

// Record / Entity: verify (all fields) and decode (required fields, uuid parse).
// Returns false on a verifier failure; *dec gets a decode status.
bool record_like(Verifier& v, size_t pos, bool entity, int* dec) {
    Table t;
    if (!visit_table(v, pos, &t)) return false;
    Str uuid, world, data;
    bool has_pos;
    double xyz[3];
    if (!field_str(v, t, R_UUID, &uuid) || !field_vec3(v, t, R_POS, &has_pos, xyz) ||
        !field_str(v, t, R_WORLD, &world) || !field_str(v, t, R_DATA, &data) || !field_bytes(v, t, R_FLEX))
        return false;
    --v.depth;
    if (*dec != WQ_DEC_OK) return true;  // first decode error wins (decode runs after verification)
    if (!uuid.present || (entity && !has_pos) || !world.present) {
        *dec = WQ_DEC_MISSING_FIELD;
        return true;
    }
    uint8_t u[16];
    if (!parse_uuid(v.b + uuid.off, uuid.len, u)) *dec = WQ_DEC_BAD_UUID;
    return true;
}

bool table_vector(Verifier& v, const Table& t, size_t voff, bool entity, uint32_t* count, int* dec) {
    size_t fp;
    *count = 0;
    if (!field(v, t, voff, &fp)) return false;
    if (!fp) return true;
    size_t vp, start, len;
    if (!v.follow(fp, &vp) || !v.aligned(vp, 4) || !v.vec_range(vp, 4, &start, &len)) return false;
    for (size_t i = 0; i < len; ++i) {
        size_t rp;
        if (!v.follow(start + 4 * i, &rp) || !record_like(v, rp, entity, dec)) return false;
    }
    *count = (uint32_t)len;
    return true;
}

void decode_one(const uint8_t* b, size_t n, wq_decoded_msg* o) {
    memset(o, 0, sizeof(*o));
    Verifier v{b, n};
    Table t;
    size_t root;
    Str param, sender, world;
    uint8_t instr = 0, repl = 0;
    bool has_pos = false;
    double xyz[3] = {0, 0, 0};
    uint32_t nrec = 0, nent = 0;
    int rec_dec = WQ_DEC_OK, ent_dec = WQ_DEC_OK;
    const bool verified = v.follow(0, &root) && visit_table(v, root, &t) &&
                          field_u8(v, t, M_INSTR, 0, &instr) && field_str(v, t, M_PARAM, &param) &&
                          field_str(v, t, M_SENDER, &sender) && field_str(v, t, M_WORLD, &world) &&
                          field_u8(v, t, M_REPL, 0, &repl) &&
                          table_vector(v, t, M_RECORDS, false, &nrec, &rec_dec) &&
                          table_vector(v, t, M_ENTITIES, true, &nent, &ent_dec) &&
                          field_vec3(v, t, M_POS, &has_pos, xyz) && field_bytes(v, t, M_FLEX);
    if (!verified || !v.ok) {
        o->status = WQ_DEC_INVALID_FLATBUFFER;
        return;
    }
    // message.rs:60-114, in its order: world_name, sender_uuid, records, entities, uuid parse
    if (!world.present || !sender.present) {
        o->status = WQ_DEC_MISSING_FIELD;
        return;
    }
    if (rec_dec != WQ_DEC_OK) {
        o->status = rec_dec;
        return;
    }
    if (ent_dec != WQ_DEC_OK) {
        o->status = ent_dec;
        return;
    }
    uint8_t u[16];
    if (!parse_uuid(b + sender.off, sender.len, u)) {
        o->status = WQ_DEC_BAD_UUID;
        return;
    }
    memcpy(o->sender_uuid, u, 16);
    o->status = WQ_DEC_OK;
    o->instruction = instr <= 12 ? instr : (uint8_t)WQ_INSTR_UNKNOWN;
    o->replication = repl <= 2 ? repl : 0;
    o->has_position = has_pos ? 1 : 0;
    o->has_parameter = param.present ? 1 : 0;
    memcpy(o->position, xyz, sizeof(xyz));
    o->world_off = world.off;
    o->world_len = world.len;
    o->param_off = param.off;
    o->param_len = param.len;
    o->n_records = nrec;
    o->n_entities = nent;
}

}  // namespace

extern "C" int wq_decode_messages(const uint8_t* data, const uint64_t* offsets, size_t n, wq_decoded_msg* out,
                                  int n_threads) {
    if (n == 0) return 0;
    if (!data || !offsets || !out) return -1;
    for (size_t i = 0; i < n; ++i)
        if (offsets[i + 1] < offsets[i]) return -1;
    size_t T = n_threads > 0 ? (size_t)n_threads : std::max(1u, std::thread::hardware_concurrency());
    T = std::min<size_t>(T, std::max<size_t>(1, n / 4096));  // a thread per >= 4k frames
    auto run = [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) decode_one(data + offsets[i], (size_t)(offsets[i + 1] - offsets[i]), out + i);
    };
    if (T <= 1) {
        run(0, n);
        return 0;
    }
    std::vector<std::thread> th;
    for (size_t k = 0; k < T; ++k) th.emplace_back(run, n * k / T, n * (k + 1) / T);
    for (auto& x : th) x.join();
    return 0;
}

extern "C" int wq_sanitize_world_name(const char* name, size_t len, char* out, size_t cap, size_t* out_len) {
    // world_names.rs:54-87, in its order of checks
    if (len == 7 && memcmp(name, "@global", 7) == 0) return WQ_SAN_IS_GLOBAL_WORLD;
    if (len == 0) return WQ_SAN_ZERO_LENGTH;
    auto alpha = [](uint8_t c) { return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z'); };
    // the first *char*: a non-ASCII lead byte is never a valid start
    if (!alpha((uint8_t)name[0])) return WQ_SAN_INVALID_START;
    size_t outn = 0;
    for (size_t i = 0; i < len; ++i) {
        const uint8_t c = (uint8_t)name[i];
        if (!(alpha(c) || (c >= '0' && c <= '9') || c == '_' || c == ' ' || c == '/' || c == '\\' || c == ':' ||
              c == '@'))
            return WQ_SAN_INVALID_CHARS;
        outn += (c == '/' || c == '\\' || c == ':' || c == '@') ? 4 : 1;
    }
    if (outn > 63) return WQ_SAN_TOO_LONG;
    if (!out || cap < outn) return -1;
    size_t k = 0;
    for (size_t i = 0; i < len; ++i) {
        const char c = name[i];
        const char* rep = c == ' ' ? "_" : c == '/' ? "_fs_" : c == '\\' ? "_bs_" : c == ':' ? "_cl_" : c == '@' ? "_at_" : nullptr;
        if (rep) {
            const size_t rl = strlen(rep);
            memcpy(out + k, rep, rl);
            k += rl;
        } else {
            out[k++] = c;
        }
    }
    if (out_len) *out_len = k;
    return 0;
}
