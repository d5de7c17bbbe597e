"""World-name validation and interning (host side of the boundary).

`sanitize_world_name` follows worldql_server/src/utils/world_names.rs:54-87: the sanitized
name is the world's identity, so distinct raw names can share a world ("a b" == "a_b").
`WorldIds` interns sanitized names to the dense u32 world ids the C ABI takes.
"""
from __future__ import annotations

GLOBAL_WORLD = "@global"  # world_names.rs:8
MAX_NAME_LENGTH = 63      # world_names.rs:51

_START = set("ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz")
_CHARSET = _START | set("0123456789_") | set(" /\\:@")
_REPLACEMENTS = ((" ", "_"), ("/", "_fs_"), ("\\", "_bs_"), (":", "_cl_"), ("@", "_at_"))


class SanitizeError(ValueError):
    """Variants of world_names.rs:89-105."""

    def __init__(self, kind: str):
        super().__init__(kind)
        self.kind = kind


def sanitize_world_name(world_name: str) -> str:
    if world_name == GLOBAL_WORLD:
        raise SanitizeError("IsGlobalWorld")
    if len(world_name) == 0:
        raise SanitizeError("ZeroLength")
    if world_name[0] not in _START:
        raise SanitizeError("InvalidStart")
    if not all(ch in _CHARSET for ch in world_name):
        raise SanitizeError("InvalidChars")
    for ch, rep in _REPLACEMENTS:  # same order as world_names.rs:76-80
        world_name = world_name.replace(ch, rep)
    if len(world_name.encode("utf-8")) > MAX_NAME_LENGTH:
        raise SanitizeError("TooLong")
    return world_name


class WorldIds:
    """Sanitized world name <-> dense u32 id (0xFFFFFFFF is reserved by the ABI)."""

    def __init__(self):
        self._ids: dict[str, int] = {}
        self._names: list[str] = []

    def get(self, sanitized: str):
        return self._ids.get(sanitized)

    def intern(self, sanitized: str) -> int:
        wid = self._ids.get(sanitized)
        if wid is None:
            wid = len(self._names)
            if wid >= 0xFFFFFFFF:
                raise OverflowError("world id space exhausted")
            self._ids[sanitized] = wid
            self._names.append(sanitized)
        return wid

    def name(self, wid: int) -> str:
        return self._names[wid]

    def __len__(self):
        return len(self._names)
