// world_map.hpp — C++ host mirror of the reference's subscription API over the C ABI.
//
// Same types, method names and return meanings as worldql_server/src/subscriptions/
// {world_map.rs:10-62, area_map.rs:10-135, cube_area.rs:8-77} and
// worldql_server/src/utils/world_names.rs:54-87, so a C++ (or, through INTEGRATION.md, Rust)
// server keeps calling WorldMap / AreaMap while the table lives on the GPU. Peers are the dense
// u32 ids of the ABI (the caller keeps its Uuid <-> u32 map). Header-only; link libwq_router.so.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "wq_router.h"

namespace worldql {

struct Vector3 {  // structures/vector3.rs:11-15
    double x, y, z;
};
struct CubeArea {  // subscriptions/cube_area.rs:8-13 (raw keys pass through unchanged)
    int64_t x, y, z;
};

class Error : public std::runtime_error {
   public:
    Error(int code, const std::string& what) : std::runtime_error(what), code(code) {}
    int code;
};

// world_names.rs:89-105
enum class SanitizeError { IsGlobalWorld, ZeroLength, InvalidStart, InvalidChars, TooLong };

inline const char* GLOBAL_WORLD = "@global";  // world_names.rs:8

// world_names.rs:54-87. Returns false and sets *err on an invalid name.
inline bool sanitize_world_name(const std::string& in, std::string* out, SanitizeError* err) {
    auto is_alpha = [](char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); };
    auto valid = [&](char c) {
        return is_alpha(c) || (c >= '0' && c <= '9') || c == '_' || c == ' ' || c == '/' || c == '\\' || c == ':' ||
               c == '@';
    };
    if (in == GLOBAL_WORLD) return *err = SanitizeError::IsGlobalWorld, false;
    if (in.empty()) return *err = SanitizeError::ZeroLength, false;
    if (!is_alpha(in[0])) return *err = SanitizeError::InvalidStart, false;
    for (char c : in)
        if (!valid(c)) return *err = SanitizeError::InvalidChars, false;
    std::string s;
    for (char c : in) {  // replacements in the reference's order give the same result per char
        switch (c) {
            case ' ': s += "_"; break;
            case '/': s += "_fs_"; break;
            case '\\': s += "_bs_"; break;
            case ':': s += "_cl_"; break;
            case '@': s += "_at_"; break;
            default: s += c;
        }
    }
    if (s.size() > 63) return *err = SanitizeError::TooLong, false;
    *out = s;
    return true;
}

class WorldMap;

// area_map.rs:10-135 — one world of the shared GPU table.
class AreaMap {
   public:
    const std::string& world_name() const { return name_; }
    uint32_t world_id() const { return id_; }

    bool is_peer_subscribed(uint32_t peer, const CubeArea& c) const { return query(peer, 1, &c.x); }
    bool is_peer_subscribed(uint32_t peer, const Vector3& v) const { return query(peer, 0, &v.x); }
    bool is_peer_subscribed_any(uint32_t peer) const;
    std::vector<uint32_t> get_subscribed_peers(const CubeArea& c) const;
    std::vector<uint32_t> get_subscribed_peers(const Vector3& v) const;
    std::vector<uint32_t> get_subscribed_any_peers() const;
    bool add_subscription(uint32_t peer, const CubeArea& c) { return mutate(peer, WQ_OP_SUBSCRIBE, c); }
    bool add_subscription(uint32_t peer, const Vector3& v) { return mutate(peer, WQ_OP_SUBSCRIBE, v); }
    bool remove_subscription(uint32_t peer, const CubeArea& c) { return mutate(peer, WQ_OP_UNSUBSCRIBE, c); }
    bool remove_subscription(uint32_t peer, const Vector3& v) { return mutate(peer, WQ_OP_UNSUBSCRIBE, v); }
    bool remove_peer(uint32_t peer);

   private:
    friend class WorldMap;
    AreaMap(WorldMap* wm, std::string name, uint32_t id) : wm_(wm), name_(std::move(name)), id_(id) {}
    bool query(uint32_t peer, int raw, const void* k) const;
    template <typename K>
    bool mutate(uint32_t peer, uint8_t kind, const K& k);
    WorldMap* wm_;
    std::string name_;
    uint32_t id_;
};

// world_map.rs:10-62
class WorldMap {
   public:
    explicit WorldMap(uint16_t cube_size, int device = 0) {
        int rc = wq_router_create(cube_size, device, &h_);
        if (rc) throw Error(rc, std::string("wq_router_create: ") + wq_last_error(nullptr));
    }
    // The same map over several GPUs behind one handle (wq_router_create_multi_mode; devices may
    // repeat): WQ_MULTI_CUBE_HASH shards the table, WQ_MULTI_REPLICATE holds it whole on each device.
    WorldMap(uint16_t cube_size, const std::vector<int>& devices, int mode = WQ_MULTI_CUBE_HASH) {
        int rc = wq_router_create_multi_mode(cube_size, (int)devices.size(), devices.data(), mode, &h_);
        if (rc) throw Error(rc, std::string("wq_router_create_multi_mode: ") + wq_last_error(nullptr));
    }
    ~WorldMap() {
        for (auto& kv : maps_) delete kv.second;
        if (h_) wq_router_destroy(h_);
    }
    WorldMap(const WorldMap&) = delete;
    WorldMap& operator=(const WorldMap&) = delete;

    AreaMap* get(const std::string& world) {  // world_map.rs:25-27
        auto it = maps_.find(world);
        return it == maps_.end() ? nullptr : it->second;
    }
    AreaMap& get_mut(const std::string& world) {  // world_map.rs:31-36
        auto it = maps_.find(world);
        if (it != maps_.end()) return *it->second;
        AreaMap* am = new AreaMap(this, world, (uint32_t)maps_.size());
        maps_.emplace(world, am);
        return *am;
    }
    bool remove_peer(uint32_t peer) {  // world_map.rs:41-61
        bool removed = false;
        for (auto& kv : maps_) removed |= kv.second->is_peer_subscribed_any(peer);
        wq_op op{};
        op.world = WQ_WORLD_INVALID;
        op.peer = peer;
        op.kind = WQ_OP_REMOVE_PEER;
        check(wq_apply_ops(h_, &op, 1));
        return removed;
    }

    // batch paths (the throughput API)
    void apply_ops(const std::vector<wq_op>& ops) { check(wq_apply_ops(h_, ops.data(), ops.size())); }
    struct Routed {
        std::vector<uint32_t> offsets, peers;
    };
    Routed route(const std::vector<double>& pos, const std::vector<uint32_t>& world, const std::vector<uint32_t>& sender,
                 const std::vector<uint8_t>& repl) {
        Routed r;
        const size_t M = world.size();
        r.offsets.resize(M + 1);
        r.peers.resize(16 * M + 64);
        size_t n = 0;
        int rc = wq_route_tick(h_, pos.data(), nullptr, world.data(), sender.data(), repl.data(), M, r.offsets.data(),
                               r.peers.data(), nullptr, r.peers.size(), &n);
        if (rc == WQ_E_CAPACITY) {
            r.peers.resize(n);
            rc = wq_route_tick(h_, pos.data(), nullptr, world.data(), sender.data(), repl.data(), M, r.offsets.data(),
                               r.peers.data(), nullptr, r.peers.size(), &n);
        }
        check(rc);
        r.peers.resize(n);
        return r;
    }
    // The scaling form over the handle's devices: slice g's messages (device pointers on device g)
    // routed there, each CSR left on its device (wq_route_tick_slices_device).
    std::vector<wq_slice_view> route_slices(const std::vector<wq_msg_slice>& slices, bool with_msgs = false) {
        std::vector<wq_slice_view> v(slices.size());
        check(wq_route_tick_slices_device(h_, slices.data(), with_msgs ? 1 : 0, v.data()));
        return v;
    }
    wq_router* handle() { return h_; }
    void check(int rc) const {
        if (rc) throw Error(rc, wq_last_error(h_));
    }

   private:
    wq_router* h_ = nullptr;
    std::unordered_map<std::string, AreaMap*> maps_;
};

inline bool AreaMap::query(uint32_t peer, int raw, const void* k) const {
    uint8_t out = 0;
    wm_->check(wq_is_subscribed(wm_->handle(), 1, &id_, &peer, raw, k, &out));
    return out != 0;
}

inline bool AreaMap::is_peer_subscribed_any(uint32_t peer) const {
    uint8_t out = 0;
    wm_->check(wq_is_subscribed_any(wm_->handle(), 1, &id_, &peer, &out));
    return out != 0;
}

template <typename K>
bool AreaMap::mutate(uint32_t peer, uint8_t kind, const K& k) {
    const bool was = is_peer_subscribed(peer, k);
    wq_op op{};
    op.world = id_;
    op.peer = peer;
    op.kind = kind;
    if constexpr (std::is_same<K, CubeArea>::value) {
        op.key_is_raw = 1;
        op.u.key[0] = k.x, op.u.key[1] = k.y, op.u.key[2] = k.z;
    } else {
        op.key_is_raw = 0;
        op.u.pos[0] = k.x, op.u.pos[1] = k.y, op.u.pos[2] = k.z;
    }
    wm_->check(wq_apply_ops(wm_->handle(), &op, 1));
    return kind == WQ_OP_SUBSCRIBE ? !was : was;  // add: newly added; remove: was present
}

inline bool AreaMap::remove_peer(uint32_t peer) {  // area_map.rs:124-135
    const bool was = is_peer_subscribed_any(peer);
    wq_op op{};
    op.world = id_;
    op.peer = peer;
    op.kind = WQ_OP_REMOVE_PEER;
    wm_->check(wq_apply_ops(wm_->handle(), &op, 1));
    return was;
}

inline std::vector<uint32_t> AreaMap::get_subscribed_peers(const CubeArea& c) const {
    const int64_t key[3] = {c.x, c.y, c.z};
    const uint32_t sender = 0;
    const uint8_t repl = WQ_REPL_INCLUDING_SELF;
    uint32_t off[2];
    std::vector<uint32_t> peers(1024);
    size_t n = 0;
    int rc = wq_route_tick(wm_->handle(), nullptr, key, &id_, &sender, &repl, 1, off, peers.data(), nullptr,
                           peers.size(), &n);
    if (rc == WQ_E_CAPACITY) {
        peers.resize(n);
        rc = wq_route_tick(wm_->handle(), nullptr, key, &id_, &sender, &repl, 1, off, peers.data(), nullptr,
                           peers.size(), &n);
    }
    wm_->check(rc);
    peers.resize(n);
    return peers;
}

inline std::vector<uint32_t> AreaMap::get_subscribed_peers(const Vector3& v) const {
    const double pos[3] = {v.x, v.y, v.z};
    const uint32_t sender = 0;
    const uint8_t repl = WQ_REPL_INCLUDING_SELF;
    uint32_t off[2];
    std::vector<uint32_t> peers(1024);
    size_t n = 0;
    int rc = wq_route_tick(wm_->handle(), pos, nullptr, &id_, &sender, &repl, 1, off, peers.data(), nullptr,
                           peers.size(), &n);
    if (rc == WQ_E_CAPACITY) {
        peers.resize(n);
        rc = wq_route_tick(wm_->handle(), pos, nullptr, &id_, &sender, &repl, 1, off, peers.data(), nullptr,
                           peers.size(), &n);
    }
    wm_->check(rc);
    peers.resize(n);
    return peers;
}

inline std::vector<uint32_t> AreaMap::get_subscribed_any_peers() const {
    size_t n = 0;
    int rc = wq_world_peers(wm_->handle(), id_, nullptr, 0, &n);
    if (rc && rc != WQ_E_CAPACITY) wm_->check(rc);
    std::vector<uint32_t> out(n);
    wm_->check(wq_world_peers(wm_->handle(), id_, out.data(), n, &n));
    return out;
}

}  // namespace worldql
