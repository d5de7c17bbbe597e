// The reference's own subscription unit tests, ported to the C++ host mirror over the C ABI:
//   area_subscriptions, world_subscriptions (worldql_server/src/subscriptions/area_map.rs:154-254),
//   sanitize (worldql_server/src/utils/world_names.rs:127-171).
// Built and run by tests/test_cpp_mirror.py (the run needs a gfx950 GPU; exit code 0 = pass).
#include <cstdio>
#include <cstdlib>
#include <string>

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

static void area_subscriptions() {
    WorldMap wm(16);
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

static void world_subscriptions() {
    const uint32_t uuid_1 = 1, uuid_2 = 2;
    const CubeArea cube_1{0, 0, 0}, cube_2{16, 16, 16};
    WorldMap wm(16);
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
    area_subscriptions();
    world_subscriptions();
    std::printf(g_fail ? "FAILED (%d)\n" : "ok\n", g_fail);
    return g_fail ? 1 : 0;
}
