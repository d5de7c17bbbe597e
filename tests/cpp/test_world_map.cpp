// The reference's own subscription unit tests, ported to the C++ host mirror over the C ABI:
//   area_subscriptions, world_subscriptions (worldql_server/src/subscriptions/area_map.rs:154-254),
//   sanitize (worldql_server/src/utils/world_names.rs:127-171).
// Built and run by tests/test_cpp_mirror.py (the run needs a gfx950 GPU; exit code 0 = pass).
#include <cstdio>
#include <exception>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "world_map.hpp"

using namespace worldql;

static int g_fail = 0;
#define CHECK(cond)                                                    \
    do {                                                               \
        if (!(cond)) {                                                 \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            ++g_fail;                                                  \
        }                                                              \
    } while (0)

// devs empty: one GPU (wq_router_create); else one handle over those devices (wq_router_create_multi_mode)
static int g_mode = WQ_MULTI_CUBE_HASH;
static WorldMap* make_map(const std::vector<int>& devs) {
    return devs.empty() ? new WorldMap(16) : new WorldMap(16, devs, g_mode);
}

static void area_subscriptions(const std::vector<int>& devs) {
    std::unique_ptr<WorldMap> wmp(make_map(devs));
    WorldMap& wm = *wmp;
    AreaMap& map = wm.get_mut("world");
    const uint32_t uuid = 7;
    const CubeArea cube_1{0, 0, 0}, cube_2{16, 16, 16};
    const Vector3 vec_1{6.3, 1.0, 10.5};  // Equivalent to cube_2
    CHECK(!map.is_peer_subscribed(uuid, cube_1));
    CHECK(!map.is_peer_subscribed(uuid, cube_2));
    CHECK(!map.is_peer_subscribed(uuid, vec_1));
    map.add_subscription(uuid, cube_1);
    CHECK(map.is_peer_subscribed(uuid, cube_1));
    CHECK(!map.is_peer_subscribed(uuid, cube_2));
    CHECK(!map.is_peer_subscribed(uuid, vec_1));
    map.add_subscription(uuid, cube_2);
    CHECK(map.is_peer_subscribed(uuid, cube_1));
    CHECK(map.is_peer_subscribed(uuid, cube_2));
    CHECK(map.is_peer_subscribed(uuid, vec_1));
    map.remove_subscription(uuid, cube_1);
    CHECK(!map.is_peer_subscribed(uuid, cube_1));
    CHECK(map.is_peer_subscribed(uuid, cube_2));
    CHECK(map.is_peer_subscribed(uuid, vec_1));
    map.remove_subscription(uuid, cube_2);
    CHECK(!map.is_peer_subscribed(uuid, cube_1));
    CHECK(!map.is_peer_subscribed(uuid, cube_2));
    CHECK(!map.is_peer_subscribed(uuid, vec_1));
    map.add_subscription(uuid, vec_1);
    CHECK(!map.is_peer_subscribed(uuid, cube_1));
    CHECK(map.is_peer_subscribed(uuid, cube_2));
    CHECK(map.is_peer_subscribed(uuid, vec_1));
    map.remove_subscription(uuid, vec_1);
    CHECK(!map.is_peer_subscribed(uuid, cube_1));
    CHECK(!map.is_peer_subscribed(uuid, cube_2));
    CHECK(!map.is_peer_subscribed(uuid, vec_1));
}

static void world_subscriptions(const std::vector<int>& devs) {
    const uint32_t uuid_1 = 1, uuid_2 = 2;
    const CubeArea cube_1{0, 0, 0}, cube_2{16, 16, 16};
    std::unique_ptr<WorldMap> wmp(make_map(devs));
    WorldMap& wm = *wmp;
    AreaMap& map = wm.get_mut("world");
    CHECK(!map.is_peer_subscribed_any(uuid_1));
    CHECK(!map.is_peer_subscribed_any(uuid_2));
    map.add_subscription(uuid_1, cube_1);
    CHECK(map.is_peer_subscribed_any(uuid_1));
    CHECK(!map.is_peer_subscribed_any(uuid_2));
    map.add_subscription(uuid_1, cube_2);
    CHECK(map.is_peer_subscribed_any(uuid_1));
    CHECK(!map.is_peer_subscribed_any(uuid_2));
    map.add_subscription(uuid_2, cube_2);
    CHECK(map.is_peer_subscribed_any(uuid_1));
    CHECK(map.is_peer_subscribed_any(uuid_2));
    map.remove_subscription(uuid_1, cube_1);
    CHECK(map.is_peer_subscribed_any(uuid_1));
    CHECK(map.is_peer_subscribed_any(uuid_2));
    map.remove_subscription(uuid_1, cube_2);
    CHECK(!map.is_peer_subscribed_any(uuid_1));
    CHECK(map.is_peer_subscribed_any(uuid_2));
    map.add_subscription(uuid_2, cube_1);
    CHECK(!map.is_peer_subscribed_any(uuid_1));
    CHECK(map.is_peer_subscribed_any(uuid_2));
    map.remove_peer(uuid_2);
    CHECK(!map.is_peer_subscribed_any(uuid_1));
    CHECK(!map.is_peer_subscribed_any(uuid_2));
}

// The batch path over the same map: messages to the neighbourhood of subscribed peers, every
// replication mode, routed through wq_route_tick; per message the recipients must be what the
// map's own membership queries say (get_subscribed_peers, then the replication filter).
static void multi_route(const std::vector<int>& devs) {
    std::unique_ptr<WorldMap> wmp(make_map(devs));
    WorldMap& wm = *wmp;
    AreaMap& map = wm.get_mut("world");
    std::vector<wq_op> ops;
    uint64_t x = 12345;
    auto rnd = [&]() { x = x * 6364136223846793005ull + 1442695040888963407ull; return (double)(x >> 11) * 0x1p-53; };
    for (uint32_t p = 0; p < 400; ++p)
        for (int k = 0; k < 3; ++k) {
            wq_op op{};
            op.world = map.world_id();
            op.peer = p;
            op.kind = WQ_OP_SUBSCRIBE;
            op.u.pos[0] = rnd() * 96 - 48, op.u.pos[1] = rnd() * 96 - 48, op.u.pos[2] = rnd() * 96 - 48;
            ops.push_back(op);
        }
    wm.apply_ops(ops);
    const size_t M = 3000;
    std::vector<double> pos(3 * M);
    std::vector<uint32_t> world(M, map.world_id()), sender(M);
    std::vector<uint8_t> repl(M);
    for (size_t i = 0; i < M; ++i) {
        for (int d = 0; d < 3; ++d) pos[3 * i + d] = rnd() * 96 - 48;
        sender[i] = (uint32_t)(rnd() * 400);
        repl[i] = (uint8_t)(rnd() * 3);
    }
    WorldMap::Routed r = wm.route(pos, world, sender, repl);
    CHECK(r.offsets.size() == M + 1 && r.offsets[M] == r.peers.size());
    size_t bad = 0;
    for (size_t i = 0; i < M && bad < 5; ++i) {
        std::vector<uint32_t> want;
        for (uint32_t p : map.get_subscribed_peers(Vector3{pos[3 * i], pos[3 * i + 1], pos[3 * i + 2]})) {
            const bool keep = repl[i] == WQ_REPL_INCLUDING_SELF ? true
                              : repl[i] == WQ_REPL_ONLY_SELF    ? p == sender[i]
                                                                : p != sender[i];
            if (keep) want.push_back(p);
        }
        const std::vector<uint32_t> got(r.peers.begin() + r.offsets[i], r.peers.begin() + r.offsets[i + 1]);
        if (got != want) ++bad;
    }
    CHECK(bad == 0);
    CHECK(r.peers.size() > M);  // the neighbourhoods overlap: plenty of recipients
}

// The scaling form: each device's own messages routed where they are (wq_route_tick_slices_device);
// every view must hold, per message, what the map's membership queries say.
static void slices_route(const std::vector<int>& devs) {
    if (devs.empty()) return;
    std::unique_ptr<WorldMap> wmp(make_map(devs));
    WorldMap& wm = *wmp;
    AreaMap& map = wm.get_mut("world");
    std::vector<wq_op> ops;
    uint64_t x = 777;
    auto rnd = [&]() { x = x * 6364136223846793005ull + 1442695040888963407ull; return (double)(x >> 11) * 0x1p-53; };
    for (uint32_t p = 0; p < 300; ++p)
        for (int k = 0; k < 3; ++k) {
            wq_op op{};
            op.world = map.world_id();
            op.peer = p;
            op.kind = WQ_OP_SUBSCRIBE;
            op.u.pos[0] = rnd() * 64 - 32, op.u.pos[1] = rnd() * 64 - 32, op.u.pos[2] = rnd() * 64 - 32;
            ops.push_back(op);
        }
    wm.apply_ops(ops);
    const size_t G = devs.size(), per = 1000;
    std::vector<std::vector<double>> pos(G, std::vector<double>(3 * per));
    std::vector<std::vector<uint32_t>> sender(G, std::vector<uint32_t>(per));
    std::vector<std::vector<uint8_t>> repl(G, std::vector<uint8_t>(per));
    std::vector<wq_msg_slice> in(G);
    std::vector<void*> bufs;
    for (size_t g = 0; g < G; ++g) {
        for (size_t i = 0; i < per; ++i) {
            for (int d = 0; d < 3; ++d) pos[g][3 * i + d] = rnd() * 64 - 32;
            sender[g][i] = (uint32_t)(rnd() * 300);
            repl[g][i] = (uint8_t)(rnd() * 3);
        }
        std::vector<uint32_t> world(per, map.world_id());
        CHECK(hipSetDevice(devs[g]) == hipSuccess);
        void *dp, *dw, *ds, *dr;
        CHECK(hipMalloc(&dp, per * 24) == hipSuccess && hipMalloc(&dw, per * 4) == hipSuccess &&
              hipMalloc(&ds, per * 4) == hipSuccess && hipMalloc(&dr, per) == hipSuccess);
        CHECK(hipMemcpy(dp, pos[g].data(), per * 24, hipMemcpyHostToDevice) == hipSuccess);
        CHECK(hipMemcpy(dw, world.data(), per * 4, hipMemcpyHostToDevice) == hipSuccess);
        CHECK(hipMemcpy(ds, sender[g].data(), per * 4, hipMemcpyHostToDevice) == hipSuccess);
        CHECK(hipMemcpy(dr, repl[g].data(), per, hipMemcpyHostToDevice) == hipSuccess);
        bufs.insert(bufs.end(), {dp, dw, ds, dr});
        in[g] = wq_msg_slice{static_cast<const double*>(dp), nullptr, static_cast<const uint32_t*>(dw),
                             static_cast<const uint32_t*>(ds), static_cast<const uint8_t*>(dr), per};
    }
    const std::vector<wq_slice_view> v = wm.route_slices(in);
    // the views point into the handle's workspace until its next call: copy every slice out first
    std::vector<std::vector<uint32_t>> all_offs(G), all_peers(G);
    for (size_t g = 0; g < G; ++g) {
        CHECK(v[g].device == devs[g] && v[g].n_msgs == per && v[g].n_pairs <= 64 * per);
        all_offs[g].resize(per + 1);
        all_peers[g].resize(v[g].n_pairs <= 64 * per ? v[g].n_pairs : 0);
        CHECK(hipSetDevice(v[g].device) == hipSuccess);
        CHECK(hipMemcpy(all_offs[g].data(), v[g].offsets, (per + 1) * 4, hipMemcpyDeviceToHost) == hipSuccess);
        if (!all_peers[g].empty())
            CHECK(hipMemcpy(all_peers[g].data(), v[g].peers, all_peers[g].size() * 4, hipMemcpyDeviceToHost) ==
                  hipSuccess);
        CHECK(all_offs[g][per] == all_peers[g].size());
    }
    size_t bad = 0, pairs = 0;
    for (size_t g = 0; g < G; ++g) {
        const std::vector<uint32_t>& offs = all_offs[g];
        const std::vector<uint32_t>& peers = all_peers[g];
        for (size_t i = 0; i < per && bad < 5; ++i) {
            if (offs[i] > offs[i + 1] || offs[i + 1] > peers.size()) {
                ++bad;
                continue;
            }
            std::vector<uint32_t> want;
            for (uint32_t p : map.get_subscribed_peers(Vector3{pos[g][3 * i], pos[g][3 * i + 1], pos[g][3 * i + 2]})) {
                const bool keep = repl[g][i] == WQ_REPL_INCLUDING_SELF ? true
                                  : repl[g][i] == WQ_REPL_ONLY_SELF    ? p == sender[g][i]
                                                                       : p != sender[g][i];
                if (keep) want.push_back(p);
            }
            const std::vector<uint32_t> got(peers.begin() + offs[i], peers.begin() + offs[i + 1]);
            if (got != want) ++bad;
        }
        pairs += peers.size();
    }
    CHECK(bad == 0);
    CHECK(pairs > G * per);
    for (void* b : bufs) (void)hipFree(b);
}

static void sanitize() {
    auto ok = [](const char* in, const char* want) {
        std::string out;
        SanitizeError e;
        return sanitize_world_name(in, &out, &e) && out == want;
    };
    auto err = [](const std::string& in, SanitizeError want) {
        std::string out;
        SanitizeError e;
        return !sanitize_world_name(in, &out, &e) && e == want;
    };
    CHECK(ok("world", "world"));
    CHECK(ok("WORLD", "WORLD"));
    CHECK(ok("world_1_2_3", "world_1_2_3"));
    CHECK(ok("world one", "world_one"));
    CHECK(ok("chat/server_1", "chat_fs_server_1"));
    CHECK(ok("chat\\server_2", "chat_bs_server_2"));
    CHECK(ok("chat:server_3", "chat_cl_server_3"));
    CHECK(ok("chat@server_4", "chat_at_server_4"));
    CHECK(ok(std::string(63, 'a').c_str(), std::string(63, 'a').c_str()));
    CHECK(err(GLOBAL_WORLD, SanitizeError::IsGlobalWorld));
    CHECK(err("", SanitizeError::ZeroLength));
    for (const char* s : {"0world", "_world", "/world", "\\world", ":world", "@world", " world", "[world", "]world"})
        CHECK(err(s, SanitizeError::InvalidStart));
    for (const char* s : {"world (two)", "world&three", "world*four", "world-four"}) CHECK(err(s, SanitizeError::InvalidChars));
    CHECK(err(std::string(64, 'a'), SanitizeError::TooLong));
}

int main(int argc, char** argv) {
    sanitize();  // host only
    if (argc > 1 && std::string(argv[1]) == "--host-only") {
        std::printf(g_fail ? "FAILED\n" : "host ok\n");
        return g_fail ? 1 : 0;
    }
    // one GPU, then one handle over G = 1, 2, 3 devices (all device 0 here), in both layouts
    const std::vector<std::vector<int>> configs = {{}, {0}, {0, 0}, {0, 0, 0}};
    for (int mode : {WQ_MULTI_CUBE_HASH, WQ_MULTI_REPLICATE}) {
        g_mode = mode;
        for (const auto& devs : configs) {
            if (mode == WQ_MULTI_REPLICATE && devs.empty()) continue;  // ran once already
            const char* step = "area_subscriptions";
            try {
                area_subscriptions(devs);
                step = "world_subscriptions";
                world_subscriptions(devs);
                step = "multi_route";
                multi_route(devs);
                step = "slices_route";
                slices_route(devs);
            } catch (const std::exception& e) {
                std::fprintf(stderr, "FAIL mode %d, %zu devices, %s: %s\n", mode, devs.size(), step, e.what());
                ++g_fail;
            }
        }
    }
    std::printf(g_fail ? "FAILED (%d)\n" : "ok\n", g_fail);
    return g_fail ? 1 : 0;
}
