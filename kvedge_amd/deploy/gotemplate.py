"""A Go text/template + Sprig subset interpreter, enough to render Helm charts offline.

SURVEY.md N23: helm/kubectl are not available in this environment, and the
reference ships no tests at all; this renderer lets the chart be rendered and
checked in CI without a cluster.  It implements the language features Helm charts
commonly use (and everything deploy/helm uses):

  actions     {{ pipeline }}  with {{- / -}} whitespace trimming, {{/* comments */}}
  control     if / else if / else / end, range (list, map, `$i, $v :=`), with, define,
              template, block-free `include`
  pipelines   cmd | cmd, parenthesised sub-pipelines, variables ($x := ..., $x = ...),
              field chains (.Values.a.b, $.Chart.Name, $v.field)
  functions   default trunc trimSuffix trimPrefix trim b64enc b64dec indent nindent quote
              squote printf replace include tpl toYaml toJson upper lower title eq ne lt le
              gt ge and or not add sub mul div mod until untilStep list dict get hasKey
              int int64 float64 toString contains hasPrefix hasSuffix required empty len
              sha256sum ternary kindIs typeOf fail coalesce join split splitList last first
              semverCompare(>=, <) regexMatch

Go semantics that matter for charts are kept: `eq` is type-strict (so a string "true"
!= bool true, reproducing the reference's quirk A.2#7 where that applies), truthiness
of empty values, `and`/`or` return operands, missing map keys render as empty.
"""
from __future__ import annotations

import base64
import hashlib
import json
import re
from typing import Any, Callable, Dict, List, Optional, Tuple

import yaml


class TemplateError(Exception):
    pass


# ---------------------------------------------------------------------------
# lexer: text / action segments with trim markers
# ---------------------------------------------------------------------------
# comments end at "*/}}" (they may contain "{{ ... }}"), actions at the first "}}"
_ACTION = re.compile(r"\{\{(-\s)?(/\*.*?\*/|.*?)(\s-)?\}\}", re.S)


def _action_end(src: str, i: int) -> int:
    """Index of the '}}' closing the action whose body starts at i (quote-aware)."""
    if src.startswith("/*", i):
        j = src.find("*/", i + 2)
        if j < 0:
            raise TemplateError("unclosed comment")
        k = src.find("}}", j + 2)
        if k < 0:
            raise TemplateError("unclosed comment action")
        return k
    n = len(src)
    while i < n:
        c = src[i]
        if c == '"':
            i += 1
            while i < n and src[i] != '"':
                i += 2 if src[i] == "\\" else 1
        elif c == "`":
            i = src.find("`", i + 1)
            if i < 0:
                raise TemplateError("unclosed raw string")
        elif src.startswith("}}", i):
            return i
        i += 1
    raise TemplateError("unclosed action")


def _segments(src: str) -> List[Tuple[str, str]]:
    out: List[Tuple[str, str]] = []
    pos = 0
    while True:
        start = src.find("{{", pos)
        if start < 0:
            break
        text = src[pos:start]
        i = start + 2
        if src.startswith("- ", i) or src.startswith("-\t", i) or src.startswith("-\n", i):
            text = text.rstrip(" \t\r\n")
            i += 2
        out.append(("text", text))
        end = _action_end(src, i)
        body = src[i:end]
        trim_right = body.endswith((" -", "\t-", "\n-"))
        if trim_right:
            body = body[:-2]
        out.append(("action", body.strip()))
        pos = end + 2
        if trim_right:
            while pos < len(src) and src[pos] in " \t\r\n":
                pos += 1
    out.append(("text", src[pos:]))
    return out


# ---------------------------------------------------------------------------
# expression tokenizer
# ---------------------------------------------------------------------------
_TOK = re.compile(r"""
    (?P<ws>\s+)|
    (?P<str>"(?:[^"\\]|\\.)*")|
    (?P<raw>`[^`]*`)|
    (?P<decl>:=)|
    (?P<assign>=)|
    (?P<pipe>\|)|
    (?P<lp>\()|(?P<rp>\))|
    (?P<comma>,)|
    (?P<num>-?\d+(?:\.\d+)?)|
    (?P<var>\$[A-Za-z0-9_]*(?:\.[A-Za-z0-9_]+)*)|
    (?P<field>(?:\.[A-Za-z0-9_]+)+|\.)|
    (?P<ident>[A-Za-z_][A-Za-z0-9_]*)
""", re.X)


def _tokenize(s: str) -> List[Tuple[str, str]]:
    toks = []
    pos = 0
    while pos < len(s):
        m = _TOK.match(s, pos)
        if not m:
            raise TemplateError(f"cannot tokenize {s[pos:]!r} in {s!r}")
        kind = m.lastgroup
        if kind == "field" and toks and toks[-1][0] == "rp" and m.start() == pos and \
                s[pos - 1] == ")":
            kind = "chain"  # (pipeline).Field — no space before the dot
            toks.append((kind, m.group("field")))
        elif kind != "ws":
            toks.append((kind, m.group(kind)))
        pos = m.end()
    return toks


# ---------------------------------------------------------------------------
# AST
# ---------------------------------------------------------------------------
class Node:
    pass


class Text(Node):
    def __init__(self, s):
        self.s = s


class Action(Node):
    def __init__(self, pipe):
        self.pipe = pipe


class If(Node):
    def __init__(self):
        self.branches: List[Tuple[Any, List[Node]]] = []  # (pipe or None for else, body)


class Range(Node):
    def __init__(self, kvars, pipe):
        self.kvars, self.pipe = kvars, pipe
        self.body: List[Node] = []
        self.else_body: List[Node] = []


class With(Node):
    def __init__(self, pipe):
        self.pipe = pipe
        self.body: List[Node] = []
        self.else_body: List[Node] = []


class TemplateCall(Node):
    def __init__(self, name, pipe):
        self.name, self.pipe = name, pipe


# pipeline = (decl_vars, decl_kind, [command]); command = [operand...]
def _parse_pipeline(toks: List[Tuple[str, str]]):
    decl, kind = [], None
    # variable declarations: $a := / $a, $b := / $a =
    for i, t in enumerate(toks):
        if t[0] in ("decl", "assign"):
            names = [x[1] for x in toks[:i] if x[0] == "var"]
            if names and all(x[0] in ("var", "comma") for x in toks[:i]):
                decl, kind = names, t[0]
                toks = toks[i + 1:]
            break
    cmds, cur, depth, buf = [], [], 0, []
    i = 0
    while i < len(toks):
        t = toks[i]
        if t[0] == "lp":
            # collect sub-pipeline
            d, j = 1, i + 1
            while j < len(toks) and d:
                if toks[j][0] == "lp":
                    d += 1
                elif toks[j][0] == "rp":
                    d -= 1
                j += 1
            if d:
                raise TemplateError("unbalanced parentheses")
            sub = _parse_pipeline(toks[i + 1:j - 1])
            # field access on a parenthesised expression: (...).Field
            if j < len(toks) and toks[j][0] == "chain":
                cur.append(("subfield", sub, toks[j][1]))
                j += 1
            else:
                cur.append(("sub", sub))
            i = j
            continue
        if t[0] == "pipe":
            cmds.append(cur)
            cur = []
        else:
            cur.append(t)
        i += 1
    if cur:
        cmds.append(cur)
    return (decl, kind, cmds)


def parse(src: str) -> Tuple[List[Node], Dict[str, List[Node]]]:
    defines: Dict[str, List[Node]] = {}
    root: List[Node] = []
    stack: List[Tuple[str, Any, List[Node]]] = [("root", None, root)]

    def body() -> List[Node]:
        return stack[-1][2]

    for kind, s in _segments(src):
        if kind == "text":
            if s:
                body().append(Text(s))
            continue
        if s.startswith("/*"):
            continue
        toks = _tokenize(s)
        if not toks:
            continue
        head = toks[0]
        word = head[1] if head[0] == "ident" else None
        if word == "if":
            n = If()
            n.branches.append((_parse_pipeline(toks[1:]), []))
            body().append(n)
            stack.append(("if", n, n.branches[-1][1]))
        elif word == "else":
            top, node, _ = stack[-1]
            if len(toks) > 1 and toks[1] == ("ident", "if"):
                if top != "if":
                    raise TemplateError("else if outside if")
                node.branches.append((_parse_pipeline(toks[2:]), []))
                stack[-1] = ("if", node, node.branches[-1][1])
            else:
                if top == "if":
                    node.branches.append((None, []))
                    stack[-1] = ("if-else", node, node.branches[-1][1])
                elif top in ("range", "with"):
                    stack[-1] = (top + "-else", node, node.else_body)
                else:
                    raise TemplateError("else outside if/range/with")
        elif word == "end":
            if len(stack) == 1:
                raise TemplateError("unexpected end")
            top, node, _ = stack.pop()
            if top == "define":
                defines[node] = _
        elif word == "range":
            rest = toks[1:]
            kvars = []
            for i, t in enumerate(rest):
                if t[0] == "decl":
                    kvars = [x[1] for x in rest[:i] if x[0] == "var"]
                    rest = rest[i + 1:]
                    break
            n = Range(kvars, _parse_pipeline(rest))
            body().append(n)
            stack.append(("range", n, n.body))
        elif word == "with":
            n = With(_parse_pipeline(toks[1:]))
            body().append(n)
            stack.append(("with", n, n.body))
        elif word == "define":
            name = json.loads(toks[1][1])
            stack.append(("define", name, []))
        elif word in ("template", "block"):
            name = json.loads(toks[1][1])
            n = TemplateCall(name, _parse_pipeline(toks[2:]) if len(toks) > 2 else None)
            body().append(n)
            if word == "block":
                stack.append(("define", name, []))
        else:
            body().append(Action(_parse_pipeline(toks)))
    if len(stack) != 1:
        raise TemplateError(f"unclosed block {stack[-1][0]}")
    return root, defines


# ---------------------------------------------------------------------------
# evaluation
# ---------------------------------------------------------------------------
class _Missing:
    def __repr__(self):
        return "<no value>"


MISSING = None  # Helm renders missing values as empty


def truthy(v) -> bool:
    if v is None or v is False:
        return False
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return v != 0
    if isinstance(v, (str, list, dict, tuple)):
        return len(v) > 0
    return True


def to_str(v) -> str:
    if v is None:
        return ""
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, float) and v.is_integer():
        return str(int(v)) if abs(v) < 1e21 else repr(v)
    if isinstance(v, dict):
        return "map[" + " ".join(f"{k}:{to_str(x)}" for k, x in sorted(v.items())) + "]"
    if isinstance(v, (list, tuple)):
        return "[" + " ".join(to_str(x) for x in v) + "]"
    return str(v)


def _go_printf(fmt: str, *args) -> str:
    out, ai, i = [], 0, 0
    while i < len(fmt):
        c = fmt[i]
        if c == "%" and i + 1 < len(fmt):
            j = i + 1
            while j < len(fmt) and fmt[j] in "0123456789.-+ #":
                j += 1
            verb = fmt[j]
            flags = fmt[i + 1:j]
            if verb == "%":
                out.append("%")
            else:
                a = args[ai] if ai < len(args) else None
                ai += 1
                if verb in "sv":
                    out.append(("%" + flags + "s") % to_str(a))
                elif verb == "q":
                    out.append(json.dumps(to_str(a)))
                elif verb == "d":
                    out.append(("%" + flags + "d") % int(a))
                elif verb in "fFeEgG":
                    out.append(("%" + flags + verb) % float(a))
                elif verb == "t":
                    out.append(to_str(bool(a)))
                elif verb in "xX":
                    out.append(("%" + flags + verb) % int(a))
                else:
                    raise TemplateError(f"printf verb %{verb} unsupported")
            i = j + 1
        else:
            out.append(c)
            i += 1
    return "".join(out)


def _indent(n, s):
    pad = " " * int(n)
    return "\n".join(pad + ln for ln in to_str(s).split("\n"))


def _to_yaml(v):
    if v is None:
        return "null"
    return yaml.safe_dump(v, default_flow_style=False, sort_keys=True).rstrip("\n")


def _eq(a, *bs):
    def same(x, y):
        if isinstance(x, bool) or isinstance(y, bool):
            return type(x) is type(y) and x == y
        if isinstance(x, (int, float)) and isinstance(y, (int, float)):
            return x == y
        if type(x) is not type(y) and not (x is None or y is None):
            raise TemplateError(f"incompatible types for comparison: {x!r} {y!r}")
        return x == y
    return any(same(a, b) for b in bs)


def _num(v):
    if isinstance(v, bool):
        raise TemplateError("bool is not a number")
    if isinstance(v, (int, float)):
        return v
    if isinstance(v, str) and re.fullmatch(r"-?\d+", v):
        return int(v)
    if isinstance(v, str):
        return float(v)
    return 0 if v is None else v


def _kind(v):
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, int):
        return "int"
    if isinstance(v, float):
        return "float64"
    if isinstance(v, str):
        return "string"
    if isinstance(v, dict):
        return "map"
    if isinstance(v, (list, tuple)):
        return "slice"
    return "invalid" if v is None else type(v).__name__


def _index(coll, *keys):
    cur = coll
    for k in keys:
        if isinstance(cur, dict):
            cur = cur.get(k)
        elif isinstance(cur, (list, tuple)):
            if not isinstance(k, int) or not 0 <= k < len(cur):
                raise TemplateError(f"index out of range: {k}")
            cur = cur[k]
        elif cur is None:
            return None
        else:
            raise TemplateError(f"can't index item of type {_kind(cur)}")
    return cur


def _semver_tuple(v: str):
    v = v.lstrip("v").split("-")[0].split("+")[0]
    parts = [int(p) for p in re.findall(r"\d+", v)][:3]
    return tuple(parts + [0] * (3 - len(parts)))


def _semver_compare(constraint: str, version: str) -> bool:
    ok = True
    for c in re.split(r"\s*,\s*|\s+", constraint.strip()):
        if not c:
            continue
        m = re.match(r"(>=|<=|>|<|=|!=|\^|~)?\s*(.*)", c)
        op, ver = m.group(1) or "=", _semver_tuple(m.group(2))
        cur = _semver_tuple(version)
        ok &= {">=": cur >= ver, "<=": cur <= ver, ">": cur > ver, "<": cur < ver,
               "=": cur == ver, "!=": cur != ver, "^": cur[0] == ver[0] and cur >= ver,
               "~": cur[:2] == ver[:2] and cur >= ver}[op]
    return ok


class Renderer:
    def __init__(self, defines: Optional[Dict[str, List[Node]]] = None, strict: bool = False):
        self.defines: Dict[str, List[Node]] = dict(defines or {})
        self.strict = strict
        self.funcs: Dict[str, Callable] = self._builtin_funcs()

    def add_source(self, src: str) -> List[Node]:
        root, defs = parse(src)
        self.defines.update(defs)
        return root

    # --- functions -------------------------------------------------------
    def _builtin_funcs(self):
        def default(d, v=None):
            return v if truthy(v) else d

        def required(msg, v=None):
            if v is None or v == "":
                raise TemplateError(msg)
            return v

        def fail(msg):
            raise TemplateError(msg)

        def dict_(*kv):
            return {kv[i]: kv[i + 1] for i in range(0, len(kv) - 1, 2)}

        def ternary(a, b, c):
            return a if truthy(c) else b

        def _set(d, k, v):  # Sprig: mutates and returns the dict
            d[k] = v
            return d

        def coalesce(*vs):
            for v in vs:
                if truthy(v):
                    return v
            return None

        f = {
            "default": default,
            "required": required,
            "fail": fail,
            "trunc": lambda n, s: to_str(s)[:int(n)] if int(n) >= 0 else to_str(s)[int(n):],
            "trimSuffix": lambda suf, s: to_str(s)[:-len(suf)] if suf and to_str(s).endswith(suf) else to_str(s),
            "trimPrefix": lambda pre, s: to_str(s)[len(pre):] if pre and to_str(s).startswith(pre) else to_str(s),
            "trim": lambda s: to_str(s).strip(),
            "b64enc": lambda s: base64.b64encode(to_str(s).encode()).decode(),
            "b64dec": lambda s: base64.b64decode(to_str(s)).decode(),
            "indent": _indent,
            "nindent": lambda n, s: "\n" + _indent(n, s),
            "quote": lambda *s: " ".join(json.dumps(to_str(x)) for x in s),
            "squote": lambda *s: " ".join("'" + to_str(x) + "'" for x in s),
            "printf": lambda fmt, *a: _go_printf(fmt, *a),
            "print": lambda *a: "".join(to_str(x) for x in a),
            "replace": lambda old, new, s: to_str(s).replace(old, new),
            "toYaml": _to_yaml,
            "toJson": lambda v: json.dumps(v, separators=(",", ":"), sort_keys=True),
            "upper": lambda s: to_str(s).upper(),
            "lower": lambda s: to_str(s).lower(),
            "title": lambda s: to_str(s).title(),
            "eq": _eq,
            "ne": lambda a, b: not _eq(a, b),
            "lt": lambda a, b: a < b,
            "le": lambda a, b: a <= b,
            "gt": lambda a, b: a > b,
            "ge": lambda a, b: a >= b,
            "not": lambda v: not truthy(v),
            "add": lambda *a: sum(_num(x) for x in a),
            "sub": lambda a, b: _num(a) - _num(b),
            "mul": lambda *a: __import__("math").prod(_num(x) for x in a),
            "div": lambda a, b: int(_num(a) // _num(b)),
            "mod": lambda a, b: _num(a) % _num(b),
            "max": lambda *a: int(max(_num(x) for x in a)),
            "min": lambda *a: int(min(_num(x) for x in a)),
            "set": _set,
            "until": lambda n: list(range(int(n))),
            "untilStep": lambda a, b, c: list(range(int(a), int(b), int(c))),
            "list": lambda *a: list(a),
            "dict": dict_,
            "get": lambda d, k: (d or {}).get(k, ""),
            "hasKey": lambda d, k: k in (d or {}),
            "int": lambda v: int(_num(v)) if v not in (None, "") else 0,
            "int64": lambda v: int(_num(v)) if v not in (None, "") else 0,
            "float64": lambda v: float(_num(v)) if v not in (None, "") else 0.0,
            "toString": to_str,
            "contains": lambda sub, s: sub in to_str(s),
            "hasPrefix": lambda p, s: to_str(s).startswith(p),
            "hasSuffix": lambda p, s: to_str(s).endswith(p),
            "empty": lambda v: not truthy(v),
            "len": lambda v: len(v) if v is not None else 0,
            "sha256sum": lambda s: hashlib.sha256(to_str(s).encode()).hexdigest(),
            "ternary": ternary,
            "kindIs": lambda k, v: _kind(v) == k,
            "typeOf": _kind,
            "coalesce": coalesce,
            "join": lambda sep, v: sep.join(to_str(x) for x in (v or [])),
            "splitList": lambda sep, s: to_str(s).split(sep),
            "index": _index,
            "first": lambda v: v[0] if v else None,
            "last": lambda v: v[-1] if v else None,
            "semverCompare": _semver_compare,
            "regexMatch": lambda rx, s: re.search(rx, to_str(s)) is not None,
        }
        return f

    # --- evaluation ------------------------------------------------------
    def _field(self, base, path: str):
        cur = base
        for part in [p for p in path.split(".") if p]:
            if isinstance(cur, dict):
                cur = cur.get(part, MISSING)
            elif cur is None:
                if self.strict:
                    raise TemplateError(f"nil pointer evaluating .{part}")
                return None
            else:
                cur = getattr(cur, part, None)
        return cur

    def _operand(self, tok, dot, vars_):
        kind = tok[0]
        if kind == "str":
            return json.loads(tok[1])
        if kind == "raw":
            return tok[1][1:-1]
        if kind == "num":
            return float(tok[1]) if "." in tok[1] else int(tok[1])
        if kind == "field":
            return dot if tok[1] == "." else self._field(dot, tok[1])
        if kind == "var":
            name, _, rest = tok[1].partition(".")
            if name not in vars_:
                raise TemplateError(f"undefined variable {name}")
            v = vars_[name]
            return self._field(v, rest) if rest else v
        if kind == "sub":
            return self._pipe(tok[1], dot, vars_)
        if kind == "subfield":
            return self._field(self._pipe(tok[1], dot, vars_), tok[2])
        if kind == "ident":
            if tok[1] == "true":
                return True
            if tok[1] == "false":
                return False
            if tok[1] == "nil":
                return None
            return self._call(tok[1], [], dot, vars_)
        raise TemplateError(f"bad operand {tok}")

    def _call(self, name, args, dot, vars_):
        if name == "include" or name == "template":
            tname = args[0]
            ctx = args[1] if len(args) > 1 else None
            return self.render_define(tname, ctx)
        if name == "tpl":
            src, ctx = args
            r = Renderer(self.defines, self.strict)
            return r.render(src, ctx)
        if name == "and":
            v = True
            for a in args:
                v = a
                if not truthy(a):
                    return a
            return v
        if name == "or":
            v = False
            for a in args:
                v = a
                if truthy(a):
                    return a
            return v
        fn = self.funcs.get(name)
        if fn is None:
            raise TemplateError(f"function {name!r} not defined")
        return fn(*args)

    def _command(self, cmd, dot, vars_, piped=None, has_piped=False):
        if not cmd:
            raise TemplateError("empty command")
        head = cmd[0]
        if head[0] == "ident" and head[1] not in ("true", "false", "nil"):
            name = head[1]
            if name in ("and", "or"):
                args = [self._operand(t, dot, vars_) for t in cmd[1:]]
            else:
                args = [self._operand(t, dot, vars_) for t in cmd[1:]]
            if has_piped:
                args.append(piped)
            return self._call(name, args, dot, vars_)
        if len(cmd) > 1 or has_piped:
            raise TemplateError(f"can't give argument to non-function {head[1] if len(head) > 1 else head}")
        return self._operand(head, dot, vars_)

    def _pipe(self, pipe, dot, vars_, declare=True):
        decl, kind, cmds = pipe
        val, has = None, False
        for c in cmds:
            val = self._command(c, dot, vars_, val, has)
            has = True
        if decl:
            for name in decl:
                vars_[name] = val
            return None if declare else val
        return val

    def _exec(self, nodes: List[Node], dot, vars_, out: List[str]):
        for n in nodes:
            if isinstance(n, Text):
                out.append(n.s)
            elif isinstance(n, Action):
                v = self._pipe(n.pipe, dot, vars_)
                if not n.pipe[0]:
                    out.append(to_str(v))
            elif isinstance(n, If):
                for cond, body in n.branches:
                    if cond is None or truthy(self._pipe(cond, dot, dict(vars_), declare=False)):
                        self._exec(body, dot, vars_, out)
                        break
            elif isinstance(n, Range):
                seq = self._pipe(n.pipe, dot, vars_, declare=False)
                items = []
                if isinstance(seq, dict):
                    items = [(k, seq[k]) for k in sorted(seq)]
                elif isinstance(seq, (list, tuple)):
                    items = list(enumerate(seq))
                elif isinstance(seq, int) and not isinstance(seq, bool):
                    items = list(enumerate(range(seq)))
                if not items:
                    self._exec(n.else_body, dot, vars_, out)
                for k, v in items:
                    vv = dict(vars_)
                    if len(n.kvars) == 1:
                        vv[n.kvars[0]] = v
                    elif len(n.kvars) == 2:
                        vv[n.kvars[0]], vv[n.kvars[1]] = k, v
                    self._exec(n.body, v, vv, out)
            elif isinstance(n, With):
                v = self._pipe(n.pipe, dot, vars_, declare=False)
                if truthy(v):
                    self._exec(n.body, v, dict(vars_), out)
                else:
                    self._exec(n.else_body, dot, vars_, out)
            elif isinstance(n, TemplateCall):
                ctx = self._pipe(n.pipe, dot, vars_, declare=False) if n.pipe else None
                out.append(self.render_define(n.name, ctx))
        return out

    def render_define(self, name: str, ctx) -> str:
        if name not in self.defines:
            raise TemplateError(f"template {name!r} not defined")
        return "".join(self._exec(self.defines[name], ctx, {"$": ctx}, []))

    def render(self, src: str, ctx) -> str:
        root = self.add_source(src)
        return "".join(self._exec(root, ctx, {"$": ctx}, []))
