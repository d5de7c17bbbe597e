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
#include <memory>
#include <new>
#include <stdexcept>
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

// ---- serialize: Message::serialize (structures/message.rs:120-134) ----------------------------
static_assert(sizeof(wq_record_in) == 96 && sizeof(wq_message_in) == 128, "codec.py mirrors these layouts");
// A restatement of the flatbuffers 2.0.0 FlatBufferBuilder (crate src/builder.rs; not vendored in
// /root/reference) as MessageT::pack drives it. The buffer fills from the back: every position below
// is a "revloc" (bytes used, counted from the end), exactly as the builder's WIPOffsets count them,
// so the finished bytes do not depend on the buffer's capacity. Padding is zero.
namespace {

constexpr size_t kMaxFrame = size_t(1) << 30;  // the builder doubles from 1024 and panics past 2^31 - 1

struct FieldLoc {
    uint32_t off;  // revloc of the field's value
    uint16_t id;   // vtable slot (VT_* constant)
};

class Builder {
  public:
    void reset() {
        if (buf_.empty()) buf_.resize(1024);  // Lazy FlatBufferBuilder::with_capacity(1024), message.rs:116-117
        head_ = buf_.size();
        min_align_ = 0;
        fields_.clear();
        vtables_.clear();
    }
    uint32_t used() const { return (uint32_t)(buf_.size() - head_); }
    const uint8_t* data() const { return buf_.data() + head_; }

    // align(len, a): zero bytes so that `len` more bytes end on an `a` boundary (builder.rs align)
    void align(size_t len, size_t a) {
        min_align_ = std::max(min_align_, a);
        pad((~(size_t(used()) + len) + 1) & (a - 1));
    }
    uint32_t push_u8(uint8_t v) {
        space(1)[0] = v;
        return used();
    }
    uint32_t push_u32(uint32_t v) {
        align(4, 4);
        memcpy(space(4), &v, 4);
        return used();
    }
    // a uoffset to the object at revloc `target`: the distance from this slot forward to it
    uint32_t push_off(uint32_t target) {
        align(4, 4);
        const uint32_t slot = used() + 4;
        const uint32_t d = slot - target;
        memcpy(space(4), &d, 4);
        return used();
    }
    uint32_t push_vec3(const double* xyz) {  // Vec3d = [u8; 24]: size 24, alignment 1
        memcpy(space(24), xyz, 24);
        return used();
    }
    // create_byte_string: NUL, bytes, length (one alignment for the whole)
    uint32_t string(const char* s, size_t n) {
        align(n + 1, 4);
        push_u8(0);
        if (n) memcpy(space(n), s, n);
        return push_u32((uint32_t)n);
    }
    uint32_t bytes(const uint8_t* s, size_t n) {  // create_vector::<u8>
        align(n, 4);
        if (n) memcpy(space(n), s, n);
        return push_u32((uint32_t)n);
    }
    uint32_t offsets(const uint32_t* t, size_t n) {  // create_vector::<WIPOffset<_>>: last item first
        align(4 * n, 4);
        for (size_t i = n; i-- > 0;) push_off(t[i]);
        return push_u32((uint32_t)n);
    }
    uint32_t start_table() { return used(); }
    void slot_off(uint16_t id, uint32_t target) { fields_.push_back({push_off(target), id}); }
    void slot_vec3(uint16_t id, const double* xyz) { fields_.push_back({push_vec3(xyz), id}); }
    void slot_u8(uint16_t id, uint8_t v, uint8_t dflt) {  // push_slot: defaults are not written
        if (v != dflt) fields_.push_back({push_u8(v), id});
    }
    // end_table = write_vtable: the soffset, then this table's vtable right below it, dropped
    // again when an identical vtable was already written in this frame.
    uint32_t end_table(uint32_t start) {
        const uint32_t obj = push_u32(0xF0F0F0F0u);
        uint16_t max_id = 0;
        for (const FieldLoc& f : fields_) max_id = std::max(max_id, f.id);
        const size_t vt_len = fields_.empty() ? 4 : (size_t)max_id + 2;
        uint8_t* vt = space(vt_len);
        memset(vt, 0, vt_len);  // absent slots read 0
        const uint16_t hdr[2] = {(uint16_t)vt_len, (uint16_t)(obj - start)};
        memcpy(vt, hdr, 4);
        for (const FieldLoc& f : fields_) {
            const uint16_t o = (uint16_t)(obj - f.off);
            memcpy(vt + f.id, &o, 2);
        }
        uint32_t vt_use = 0;
        bool dup = false;
        for (size_t k = vtables_.size(); k-- > 0;) {
            const uint8_t* other = buf_.data() + buf_.size() - vtables_[k];
            uint16_t ol;
            memcpy(&ol, other, 2);
            if (ol == vt_len && memcmp(other, vt, vt_len) == 0) {
                vt_use = vtables_[k];
                dup = true;
                break;
            }
        }
        if (dup) {
            memset(vt, 0, vt_len);
            head_ += vt_len;
        } else {
            vt_use = used();
            vtables_.push_back(vt_use);
        }
        const int32_t so = (int32_t)vt_use - (int32_t)obj;
        memcpy(buf_.data() + buf_.size() - obj, &so, 4);
        fields_.clear();
        return obj;
    }
    void finish(uint32_t root) {
        vtables_.clear();
        align(4, min_align_);
        push_off(root);
    }

  private:
    std::vector<uint8_t> buf_;
    size_t head_ = 0, min_align_ = 0;
    std::vector<FieldLoc> fields_;
    std::vector<uint32_t> vtables_;

    void pad(size_t n) {
        if (n) memset(space(n), 0, n);
    }
    uint8_t* space(size_t n) {
        if (head_ < n) grow(n);
        head_ -= n;
        return buf_.data() + head_;
    }
    void grow(size_t n) {  // grow_owned_buf: double, keep the used bytes at the end
        const size_t active = used();
        size_t len = buf_.size();
        while (len - active < n) len *= 2;
        if (len > kMaxFrame) throw std::length_error("frame");
        std::vector<uint8_t> nb(len);
        memcpy(nb.data() + len - active, buf_.data() + head_, active);
        buf_.swap(nb);
        head_ = len - active;
    }
};

// Message vtable slots (WorldQLFB_generated.rs:939-947) and Record / Entity (:485-489, :704-708)
enum : uint16_t { S_INSTR = 4, S_PARAM = 6, S_SENDER = 8, S_WORLD = 10, S_REPL = 12, S_RECORDS = 14,
                  S_ENTITIES = 16, S_POS = 18, S_FLEX = 20 };
enum : uint16_t { SR_UUID = 4, SR_POS = 6, SR_WORLD = 8, SR_DATA = 10, SR_FLEX = 12 };

// uuid 0.8.2 Display: lower-case hyphenated
void uuid_text(const uint8_t u[16], char out[36]) {
    static const char* hex = "0123456789abcdef";
    int k = 0;
    for (int i = 0; i < 16; ++i) {
        if (i == 4 || i == 6 || i == 8 || i == 10) out[k++] = '-';
        out[k++] = hex[u[i] >> 4];
        out[k++] = hex[u[i] & 15];
    }
}

bool utf8_ok(const char* s, uint64_t n) { return n == 0 || (s && valid_utf8((const uint8_t*)s, n)); }

int check_record(const wq_record_in& r) {
    if (!utf8_ok(r.world_name, r.world_len) || (r.has_data && !utf8_ok(r.data, r.data_len))) return WQ_SER_INVALID_UTF8;
    if (r.has_flex && r.flex_len && !r.flex) return WQ_SER_INVALID_ARG;
    return 0;
}

// RecordT / EntityT::pack (WorldQLFB_generated.rs:619-645, :838-864) of Record / Entity::encode
// (record.rs:18-26, entity.rs:17-25): uuid, world_name, data, flex; then create() adds
// flex, data, world_name, position, uuid (:449-457, :668-676).
uint32_t pack_record(Builder& b, const wq_record_in& r, bool entity) {
    char u[36];
    uuid_text(r.uuid, u);
    const uint32_t uuid = b.string(u, 36);
    const uint32_t world = b.string(r.world_name, r.world_len);
    const uint32_t data = r.has_data ? b.string(r.data, r.data_len) : 0;
    const uint32_t flex = r.has_flex ? b.bytes(r.flex, r.flex_len) : 0;
    const uint32_t t = b.start_table();
    if (r.has_flex) b.slot_off(SR_FLEX, flex);
    if (r.has_data) b.slot_off(SR_DATA, data);
    b.slot_off(SR_WORLD, world);
    if (entity || r.has_position) b.slot_vec3(SR_POS, r.position);
    b.slot_off(SR_UUID, uuid);
    return b.end_table(t);
}

int check_message(const wq_message_in& m) {
    if (!utf8_ok(m.world_name, m.world_len) || (m.has_parameter && !utf8_ok(m.parameter, m.parameter_len)))
        return WQ_SER_INVALID_UTF8;
    if ((m.n_records && !m.records) || (m.n_entities && !m.entities) || (m.has_flex && m.flex_len && !m.flex))
        return WQ_SER_INVALID_ARG;
    for (uint64_t i = 0; i < m.n_records; ++i)
        if (int e = check_record(m.records[i])) return e;
    for (uint64_t i = 0; i < m.n_entities; ++i)
        if (int e = check_record(m.entities[i])) return e;
    return 0;
}

// MessageT::pack (WorldQLFB_generated.rs:1133-1173) of Message::encode (message.rs:28-52), then
// finish(root, None). Returns 0 with the frame at b.data()[0 .. b.used()), or an error.
int serialize_one(Builder& b, const wq_message_in& m, std::vector<uint32_t>& scratch) {
    if (int e = check_message(m)) return e;
    b.reset();
    const uint32_t param = m.has_parameter ? b.string(m.parameter, m.parameter_len) : 0;
    char u[36];
    uuid_text(m.sender_uuid, u);
    const uint32_t sender = b.string(u, 36);
    const uint32_t world = b.string(m.world_name, m.world_len);
    scratch.resize(std::max(m.n_records, m.n_entities));
    for (uint64_t i = 0; i < m.n_records; ++i) scratch[i] = pack_record(b, m.records[i], false);
    const uint32_t records = b.offsets(scratch.data(), m.n_records);  // Some(vec![]) when empty
    for (uint64_t i = 0; i < m.n_entities; ++i) scratch[i] = pack_record(b, m.entities[i], true);
    const uint32_t entities = b.offsets(scratch.data(), m.n_entities);
    const uint32_t flex = m.has_flex ? b.bytes(m.flex, m.flex_len) : 0;
    // Message::create (WorldQLFB_generated.rs:1045-1055)
    const uint32_t t = b.start_table();
    if (m.has_flex) b.slot_off(S_FLEX, flex);
    if (m.has_position) b.slot_vec3(S_POS, m.position);
    b.slot_off(S_ENTITIES, entities);
    b.slot_off(S_RECORDS, records);
    b.slot_off(S_WORLD, world);
    b.slot_off(S_SENDER, sender);
    if (m.has_parameter) b.slot_off(S_PARAM, param);
    b.slot_u8(S_REPL, m.replication, 0);   // default ExceptSelf
    b.slot_u8(S_INSTR, m.instruction, 0);  // default Heartbeat
    b.finish(b.end_table(t));
    return 0;
}

int serialize_guarded(Builder& b, const wq_message_in& m, std::vector<uint32_t>& scratch) {
    try {
        return serialize_one(b, m, scratch);
    } catch (const std::length_error&) {
        return WQ_SER_TOO_LARGE;
    } catch (const std::bad_alloc&) {
        return WQ_SER_TOO_LARGE;
    }
}

// Upper bound of a frame's size: strings NUL + length + 3 pad, byte vectors length + 3 pad, the
// Message table (soffset, 7 uoffsets, Vec3d, 2 scalars, pad) and vtable (22), root + finish pad;
// a Record / Entity table (soffset, 4 uoffsets, Vec3d, pad), vtable (14) and vector entry.
size_t frame_bound(const wq_message_in& m) {
    auto str = [](uint64_t n) { return (size_t)n + 8; };
    auto vec = [](uint64_t n) { return (size_t)n + 7; };
    size_t b = 7 + 22 + 61 + str(36) + str(m.world_len) + (m.has_parameter ? str(m.parameter_len) : 0) +
               (m.has_flex ? vec(m.flex_len) : 0) + 2 * 7;
    auto rec = [&](const wq_record_in& r) {
        return 14 + 47 + 4 + str(36) + str(r.world_len) + (r.has_data ? str(r.data_len) : 0) +
               (r.has_flex ? vec(r.flex_len) : 0);
    };
    for (uint64_t i = 0; i < m.n_records; ++i) b += rec(m.records[i]);
    for (uint64_t i = 0; i < m.n_entities; ++i) b += rec(m.entities[i]);
    return b;
}

}  // namespace

extern "C" int wq_serialize_message(const wq_message_in* m, uint8_t* out, size_t cap, size_t* out_len) {
    if (!m || !out_len) return WQ_SER_INVALID_ARG;
    // one builder per calling thread, reused across calls like the reference's global builder
    // (message.rs:116-117); looked up once per call
    static thread_local Builder tl_builder;
    static thread_local std::vector<uint32_t> tl_scratch;
    Builder& b = tl_builder;
    if (int e = serialize_guarded(b, *m, tl_scratch)) return e;
    *out_len = b.used();
    if (cap < *out_len) return WQ_SER_SHORT;
    if (!out) return WQ_SER_INVALID_ARG;
    memcpy(out, b.data(), *out_len);
    return 0;
}

extern "C" size_t wq_serialize_bound(const wq_message_in* msgs, size_t n) {
    size_t b = 0;
    for (size_t i = 0; msgs && i < n; ++i) b += frame_bound(msgs[i]);
    return b;
}

extern "C" int wq_serialize_messages(const wq_message_in* msgs, size_t n, uint8_t* out, size_t cap,
                                     uint64_t* offsets, int n_threads) {
    if (!offsets || (n && !msgs)) return WQ_SER_INVALID_ARG;
    offsets[0] = 0;
    if (n == 0) return 0;
    size_t T = n_threads > 0 ? (size_t)n_threads : std::max(1u, std::thread::hardware_concurrency());
    T = std::min<size_t>(T, std::max<size_t>(1, n / 2048));  // a thread per >= 2k frames
    auto run = [&](auto&& fn) {
        if (T == 1) {
            fn(0);
            return;
        }
        std::vector<std::thread> th;
        for (size_t k = 0; k < T; ++k) th.emplace_back(fn, k);
        for (auto& x : th) x.join();
    };
    // Worker k packs frames [n k / T, n (k + 1) / T) back to back into its own region: straight
    // into out at its bound prefix when out holds every bound (then the regions are slid down
    // into place, in order), else into an arena sized from the bounds and copied afterwards.
    std::vector<size_t> bound(T + 1, 0), used(T, 0);
    run([&](size_t k) {
        for (size_t i = n * k / T, hi = n * (k + 1) / T; i < hi; ++i) bound[k + 1] += frame_bound(msgs[i]);
    });
    for (size_t k = 0; k < T; ++k) bound[k + 1] += bound[k];
    const bool direct = out && cap >= bound[T];
    std::vector<std::unique_ptr<uint8_t[]>> arena(direct ? 0 : T);
    std::vector<int> err(T, 0);
    run([&](size_t k) {
        uint8_t* dst;
        if (direct) {
            dst = out + bound[k];
        } else {
            arena[k].reset(new uint8_t[bound[k + 1] - bound[k] + 1]);
            dst = arena[k].get();
        }
        Builder b;
        std::vector<uint32_t> scratch;
        size_t u = 0;
        for (size_t i = n * k / T, hi = n * (k + 1) / T; i < hi; ++i) {
            if (int e = serialize_guarded(b, msgs[i], scratch)) {
                err[k] = e;
                return;
            }
            memcpy(dst + u, b.data(), b.used());
            u += b.used();
            offsets[i + 1] = b.used();
        }
        used[k] = u;
    });
    for (size_t k = 0; k < T; ++k)
        if (err[k]) return err[k];  // ranges are in order: the first failing message's code
    for (size_t i = 0; i < n; ++i) offsets[i + 1] += offsets[i];
    if (direct) {
        for (size_t k = 1; k < T; ++k)  // in order: region k only moves down, over bytes already placed or free
            if (used[k]) memmove(out + offsets[n * k / T], out + bound[k], used[k]);
        return 0;
    }
    if (offsets[n] > cap) return WQ_SER_SHORT;
    if (!out) return WQ_SER_INVALID_ARG;
    run([&](size_t k) {
        if (used[k]) memcpy(out + offsets[n * k / T], arena[k].get(), used[k]);
    });
    return 0;
}
