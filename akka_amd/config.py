"""A small HOCON subset (typesafe-config 1.4.0 semantics for what dispatch needs).

Supports: nested objects `a { b = 1 }`, dotted keys `a.b.c = x`, `=`/`:`
separators, quoted and unquoted strings, integers, booleans, `#` and `//`
comments, object merging of repeated keys, and `with_fallback`.  Durations
("10ms", "0s", "1 second") are kept as strings and parsed by `get_duration`.
Used to resolve dispatcher / mailbox ids the way
akka-actor/src/main/scala/akka/dispatch/Dispatchers.scala:121-262 and
Mailboxes.scala:140-260 do.
"""
from __future__ import annotations

import copy
import re


class ConfigurationException(Exception):
    """akka.ConfigurationException"""


_TOKEN = re.compile(r'\s*("(?:[^"\\]|\\.)*"|[{}\[\],=:]|\n|[^\s{}\[\],=:#"]+(?:[ \t]+[^\s{}\[\],=:#"]+)*)')


def _strip_comments(text: str) -> str:
    out = []
    for line in text.splitlines():
        res, q = [], False
        i = 0
        while i < len(line):
            ch = line[i]
            if ch == '"' and (i == 0 or line[i - 1] != "\\"):
                q = not q
            if not q and (ch == "#" or line.startswith("//", i)):
                break
            res.append(ch)
            i += 1
        out.append("".join(res))
    return "\n".join(out)


def _tokens(text: str):
    text = _strip_comments(text)
    pos = 0
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m or m.end() == pos:
            if text[pos:].strip() == "":
                break
            raise ConfigurationException(f"HOCON parse error near: {text[pos:pos + 30]!r}")
        pos = m.end()
        yield m.group(1)


def _scalar(tok: str):
    if tok.startswith('"'):
        return bytes(tok[1:-1], "utf-8").decode("unicode_escape")
    if re.fullmatch(r"-?\d+", tok):
        return int(tok)
    if re.fullmatch(r"-?\d+\.\d+", tok):
        return float(tok)
    if tok in ("true", "on", "yes"):
        return True
    if tok in ("false", "off", "no"):
        return False
    if tok == "null":
        return None
    return tok


def _merge(dst: dict, src: dict) -> dict:
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


def _set_path(obj: dict, path: list, value):
    for p in path[:-1]:
        nxt = obj.get(p)
        if not isinstance(nxt, dict):
            nxt = {}
            obj[p] = nxt
        obj = nxt
    last = path[-1]
    if isinstance(value, dict) and isinstance(obj.get(last), dict):
        _merge(obj[last], value)
    else:
        obj[last] = value


def _split_key(tok: str) -> list:
    if tok.startswith('"'):
        return [tok[1:-1]]
    return [p.strip('"') for p in tok.split(".")]


def _parse_object(toks: list, i: int, closing: str | None):
    obj: dict = {}
    while i < len(toks):
        t = toks[i]
        if t in ("\n", ","):
            i += 1
            continue
        if t == closing:
            return obj, i + 1
        key = _split_key(t)
        i += 1
        while i < len(toks) and toks[i] == "\n":
            i += 1
        if i < len(toks) and toks[i] in ("=", ":"):
            i += 1
        while i < len(toks) and toks[i] == "\n":
            i += 1
        if i >= len(toks):
            raise ConfigurationException(f"missing value for {'.'.join(key)}")
        v = toks[i]
        if v == "{":
            val, i = _parse_object(toks, i + 1, "}")
        elif v == "[":
            val, i = _parse_list(toks, i + 1)
        else:
            val = _scalar(v)
            i += 1
        _set_path(obj, key, val)
    if closing is not None:
        raise ConfigurationException("unbalanced braces")
    return obj, i


def _parse_list(toks: list, i: int):
    out = []
    while i < len(toks):
        t = toks[i]
        if t in ("\n", ","):
            i += 1
            continue
        if t == "]":
            return out, i + 1
        if t == "{":
            v, i = _parse_object(toks, i + 1, "}")
            out.append(v)
        else:
            out.append(_scalar(t))
            i += 1
    raise ConfigurationException("unbalanced brackets")


_DUR = {"ns": 1e-9, "nanosecond": 1e-9, "nanoseconds": 1e-9, "us": 1e-6, "microsecond": 1e-6,
        "microseconds": 1e-6, "ms": 1e-3, "millisecond": 1e-3, "milliseconds": 1e-3, "s": 1.0, "second": 1.0,
        "seconds": 1.0, "m": 60.0, "minute": 60.0, "minutes": 60.0, "h": 3600.0, "hour": 3600.0, "hours": 3600.0,
        "d": 86400.0, "day": 86400.0, "days": 86400.0}


class Config:
    def __init__(self, root: dict | None = None):
        self.root = root or {}

    @classmethod
    def parse_string(cls, text: str) -> "Config":
        obj, _ = _parse_object(list(_tokens(text)), 0, None)
        return cls(obj)

    def with_fallback(self, other: "Config") -> "Config":
        merged = _merge(copy.deepcopy(other.root), self.root)
        return Config(merged)

    def _get(self, path: str):
        cur = self.root
        for p in path.split("."):
            if not isinstance(cur, dict) or p not in cur:
                raise KeyError(path)
            cur = cur[p]
        return cur

    def has_path(self, path: str) -> bool:
        try:
            return self._get(path) is not None
        except KeyError:
            return False

    def get_value(self, path: str):
        try:
            return self._get(path)
        except KeyError:
            raise ConfigurationException(f"No configuration setting found for key '{path}'") from None

    def get_config(self, path: str) -> "Config":
        v = self.get_value(path)
        if not isinstance(v, dict):
            raise ConfigurationException(f"{path} is not an object")
        return Config(v)

    def get_string(self, path: str) -> str:
        return str(self.get_value(path))

    def get_int(self, path: str) -> int:
        v = self.get_value(path)
        if isinstance(v, bool) or not isinstance(v, (int, float)):
            try:
                return int(str(v))
            except ValueError:
                raise ConfigurationException(f"{path} is not a number: {v!r}") from None
        return int(v)

    def get_duration_s(self, path: str) -> float:
        v = self.get_value(path)
        if isinstance(v, (int, float)) and not isinstance(v, bool):
            return float(v) / 1000.0  # bare numbers are milliseconds
        m = re.fullmatch(r"\s*(-?\d+(?:\.\d+)?)\s*([a-zA-Z]*)\s*", str(v))
        if not m:
            raise ConfigurationException(f"{path} is not a duration: {v!r}")
        unit = m.group(2) or "ms"
        if unit not in _DUR:
            raise ConfigurationException(f"{path}: unknown duration unit {unit!r}")
        return float(m.group(1)) * _DUR[unit]
