"""Offline TypeScript -> JavaScript (ES modules) type eraser for the reference merge-tree sources.

TEST INFRASTRUCTURE: this container has Node 12 but no `tsc`, no
`node_modules` and a Node without `?.`/`??`. To pin the engine's collaborative results to the
reference itself, the ~22 `packages/dds/merge-tree/src/*.ts` files are type-erased into a scratch
directory OUTSIDE the repository (default /tmp/mt-oracle/), never committed and never shipped, and
run by `tools/ref_replay.mjs` to produce golden vectors (`tools/make_ref_goldens.py`).

It handles exactly the TypeScript subset those files use (counted in SURVEY.md §8(c)):
  - type annotations on variables, parameters, return types, class members;
  - generic parameter / argument lists, `as T` and `<T>expr` assertions, non-null `x!`;
  - interfaces, type aliases, `declare`, overload and abstract member signatures (dropped);
  - access modifiers, `readonly`, `abstract`, `implements`; constructor parameter properties and
    instance field initializers become assignments at the top of the constructor (after
    `super(...)`), in TypeScript's order;
  - `enum` / `const enum` become frozen-order objects with TypeScript's reverse mapping;
  - `import`s of type-only names are dropped (Node's ESM loader rejects missing named exports),
    specifiers get `.mjs`, `@fluidframework/*` resolve to small shims;
  - the few `?.` / `??` uses are lowered by exact textual patches (PATCHES), not generically.
The output is checked with `node --check` by the driver script; anything unexpected raises.
"""
from __future__ import annotations

import argparse
import os
import re
import sys
from dataclasses import dataclass
from typing import Dict, List, Optional, Set, Tuple

PUNCT = sorted("""
>>>= ... === !== **= <<= >>= => == != <= >= && || ?? ?. ++ -- += -= *= /= %= &= |= ^= ** <<
{ } ( ) [ ] ; , < > + - * / % & | ^ ! ~ ? : = . @ #
""".split(), key=len, reverse=True)

KEYWORDS_BEFORE_EXPR = {"return", "typeof", "instanceof", "in", "of", "new", "delete", "void", "throw",
                        "case", "do", "else", "yield", "await", "extends"}
TS_ONLY_MODIFIERS = {"public", "private", "protected", "readonly", "abstract", "override", "declare"}
MEMBER_MODIFIERS = TS_ONLY_MODIFIERS | {"static", "async", "get", "set"}


@dataclass
class Tok:
    kind: str  # id, num, str, tmpl, re, p
    text: str
    start: int
    end: int


class EraseError(RuntimeError):
    pass


def tokenize(src: str) -> List[Tok]:
    toks: List[Tok] = []
    i, n = 0, len(src)

    def prev_ends_operand() -> bool:
        for t in reversed(toks):
            if t.kind in ("num", "str", "tmpl", "re"):
                return True
            if t.kind == "id":
                return t.text not in KEYWORDS_BEFORE_EXPR
            return t.text in (")", "]", "}")
        return False

    while i < n:
        c = src[i]
        if c in " \t\r\n﻿":
            i += 1
            continue
        if src.startswith("//", i):
            j = src.find("\n", i)
            i = n if j < 0 else j
            continue
        if src.startswith("/*", i):
            j = src.find("*/", i + 2)
            if j < 0:
                raise EraseError("unterminated comment")
            i = j + 2
            continue
        if c.isalpha() or c in "_$":
            m = re.compile(r"[A-Za-z_$][\w$]*").match(src, i)
            toks.append(Tok("id", m.group(0), i, m.end()))
            i = m.end()
            continue
        if c.isdigit() or (c == "." and i + 1 < n and src[i + 1].isdigit()):
            m = re.compile(r"0[xXbBoO][0-9a-fA-F_]+n?|(\d[\d_]*)?\.?\d*([eE][+-]?\d+)?n?").match(src, i)
            toks.append(Tok("num", m.group(0), i, m.end()))
            i = m.end()
            continue
        if c in "'\"":
            j = i + 1
            while src[j] != c:
                j += 2 if src[j] == "\\" else 1
            toks.append(Tok("str", src[i:j + 1], i, j + 1))
            i = j + 1
            continue
        if c == "`":
            j = _skip_template(src, i)
            toks.append(Tok("tmpl", src[i:j], i, j))
            i = j
            continue
        if c == "/" and not prev_ends_operand():
            j = i + 1
            in_class = False
            while True:
                ch = src[j]
                if ch == "\\":
                    j += 2
                    continue
                if ch == "[":
                    in_class = True
                elif ch == "]":
                    in_class = False
                elif ch == "/" and not in_class:
                    break
                elif ch == "\n":
                    raise EraseError(f"bad regex at {i}")
                j += 1
            j += 1
            while j < n and (src[j].isalnum()):
                j += 1
            toks.append(Tok("re", src[i:j], i, j))
            i = j
            continue
        for p in PUNCT:
            if src.startswith(p, i):
                # `>` is always one token: generic lists close with `>>`; `?.` followed by a digit is `?` `.5`
                if p[0] == ">" and p not in (">=", ">>=", ">>>="):
                    p = ">"
                if p == "?." and i + 2 < n and src[i + 2].isdigit():
                    p = "?"
                toks.append(Tok("p", p, i, i + len(p)))
                i += len(p)
                break
        else:
            raise EraseError(f"unexpected character {c!r} at {i}")
    return toks


def _skip_template(src: str, i: int) -> int:
    j = i + 1
    while True:
        ch = src[j]
        if ch == "\\":
            j += 2
            continue
        if ch == "`":
            return j + 1
        if src.startswith("${", j):
            depth = 1
            j += 2
            while depth:
                ch = src[j]
                if ch in "'\"":
                    k = j + 1
                    while src[k] != ch:
                        k += 2 if src[k] == "\\" else 1
                    j = k + 1
                    continue
                if ch == "`":
                    j = _skip_template(src, j)
                    continue
                if ch == "{":
                    depth += 1
                elif ch == "}":
                    depth -= 1
                j += 1
            continue
        j += 1


class Module:
    """One TS source file: tokens, bracket matches, edits, and its import/export statements."""

    def __init__(self, name: str, src: str):
        self.name = name
        self.src = src
        self.toks = tokenize(src)
        self.n = len(self.toks)
        self.match = self._match()
        self.dropped: Set[int] = set()
        self.repl: Dict[int, str] = {}
        self.ins_before: Dict[int, List[str]] = {}
        self.ins_after: Dict[int, List[str]] = {}
        self.local_values: Set[str] = set()  # runtime bindings declared at top level
        self.exports: Set[str] = set()  # runtime names exported (direct)
        self.star_from: List[str] = []  # export * from
        self.reexports: List[Tuple[str, List[Tuple[str, str]], Tuple[int, int]]] = []  # (spec, [(orig, as)], range)
        self.local_exports: List[Tuple[List[Tuple[str, str]], Tuple[int, int]]] = []  # export { a as b }
        self.extra_uses: Set[str] = set()  # identifiers of moved field initializers
        self.imports: List[Tuple[str, Optional[str], Optional[str], List[Tuple[str, str]], Tuple[int, int]]] = []
        # (spec, default, namespace, named [(orig, local)], token range)

    def _match(self) -> List[int]:
        m = [-1] * self.n
        st: List[int] = []
        pairs = {")": "(", "]": "[", "}": "{"}
        for i, t in enumerate(self.toks):
            if t.kind != "p":
                continue
            if t.text in ("(", "[", "{"):
                st.append(i)
            elif t.text in pairs:
                if not st or self.toks[st[-1]].text != pairs[t.text]:
                    raise EraseError(f"{self.name}: unbalanced {t.text} at {t.start}")
                j = st.pop()
                m[i] = j
                m[j] = i
        if st:
            raise EraseError(f"{self.name}: unclosed bracket")
        return m

    # ---- token helpers -------------------------------------------------------------------
    def t(self, i: int) -> str:
        return self.toks[i].text if 0 <= i < self.n else ""

    def is_id(self, i: int) -> bool:
        return 0 <= i < self.n and self.toks[i].kind == "id"

    def drop(self, a: int, b: int) -> None:
        self.dropped.update(range(a, b))

    def render(self, a: int = 0, b: Optional[int] = None) -> str:
        b = self.n if b is None else b
        out = []
        prev = self.toks[a - 1].end if a > 0 else 0
        for i in range(a, b):
            tk = self.toks[i]
            out.append(self.src[prev:tk.start])
            out.extend(self.ins_before.get(i, []))
            if i not in self.dropped:
                out.append(self.repl.get(i, tk.text))
            out.extend(self.ins_after.get(i, []))
            prev = tk.end
        if b == self.n:
            out.append(self.src[prev:])
        return "".join(out)

    def ends_operand(self, i: int) -> bool:
        if i < 0:
            return False
        tk = self.toks[i]
        if tk.kind in ("num", "str", "tmpl", "re"):
            return True
        if tk.kind == "id":
            return tk.text not in KEYWORDS_BEFORE_EXPR
        return tk.text in (")", "]")

    # ---- types ---------------------------------------------------------------------------
    def skip_type_args(self, i: int) -> int:
        """i at `<`: index after the matching `>` (generic parameter or argument list)."""
        assert self.t(i) == "<"
        depth = 0
        while i < self.n:
            x = self.t(i)
            if x == "<":
                depth += 1
            elif x == ">":
                depth -= 1
                if depth == 0:
                    return i + 1
            elif x in ("(", "[", "{"):
                i = self.match[i]
            elif x in (";", ")", "]", "}"):
                raise EraseError(f"{self.name}: bad type argument list at {self.toks[i].start}")
            i += 1
        raise EraseError("unterminated type arguments")

    def try_type_args(self, i: int) -> int:
        """Like skip_type_args but returns -1 if tokens from i are not a type-argument list."""
        depth = 0
        j = i
        while j < self.n:
            x = self.t(j)
            tk = self.toks[j]
            if x == "<":
                depth += 1
            elif x == ">":
                depth -= 1
                if depth == 0:
                    return j + 1
            elif x in ("(", "[", "{"):
                j = self.match[j]
            elif tk.kind == "id" or tk.kind == "str" or tk.kind == "num" or x in (",", ".", "|", "&", "=>", "?", ":"):
                pass
            else:
                return -1
            j += 1
        return -1

    def skip_type(self, i: int) -> int:
        """Index after the type expression starting at i."""
        if self.t(i) in ("|", "&"):
            i += 1
        i = self._type_postfix(i)
        while self.t(i) in ("|", "&"):
            i = self._type_postfix(i + 1)
        # conditional type: A extends B ? C : D
        if self.t(i) == "extends":
            i = self.skip_type(i + 1)
            if self.t(i) == "?":
                i = self.skip_type(i + 1)
                if self.t(i) != ":":
                    raise EraseError("bad conditional type")
                i = self.skip_type(i + 1)
        return i

    def _type_postfix(self, i: int) -> int:
        i = self._type_primary(i)
        while self.t(i) == "[":
            i = self.match[i] + 1
        return i

    def _type_primary(self, i: int) -> int:
        x = self.t(i)
        tk = self.toks[i]
        if x in ("keyof", "readonly", "unique", "infer") and self.toks[i + 1].kind in ("id",) or x in ("keyof", "readonly") and self.t(i + 1) in ("(", "[", "{"):
            return self._type_primary(i + 1) if x != "infer" else i + 2
        if x == "typeof":
            i += 1
            while self.is_id(i) and self.t(i + 1) == ".":
                i += 2
            return i + 1
        if x == "new":
            return self._type_primary(i + 1)
        if x == "<":  # generic function type
            i = self.skip_type_args(i)
            return self._type_primary(i)
        if x == "(":
            j = self.match[i] + 1
            if self.t(j) == "=>":
                return self.skip_type(j + 1)
            return j
        if x in ("{", "["):
            return self.match[i] + 1
        if x == "-" and self.toks[i + 1].kind == "num":
            return i + 2
        if tk.kind in ("str", "num", "tmpl"):
            return i + 1
        if tk.kind == "id":
            i += 1
            while self.t(i) == "." and self.is_id(i + 1):
                i += 2
            if self.t(i) == "<":
                i = self.skip_type_args(i)
            if self.t(i) == "is" and tk.text not in ("typeof",):  # type predicate `x is T`
                return self.skip_type(i + 1)
            return i
        raise EraseError(f"{self.name}: cannot parse type at {tk.start}: {x!r}")

    # ---- parameters ----------------------------------------------------------------------
    def params(self, a: int, b: int, ctor: bool = False) -> List[str]:
        """Erase types in the parameter list between tokens a=( and b=). Returns the names of
        constructor parameter properties."""
        props: List[str] = []
        i = a + 1
        first = True
        while i < b:
            start = i
            mods = []
            while self.t(i) in TS_ONLY_MODIFIERS and (self.is_id(i + 1) or self.t(i + 1) in ("{", "[")):
                mods.append(i)
                i += 1
            for m in mods:
                self.dropped.add(m)
            if first and self.t(i) == "this" and self.t(i + 1) == ":":
                end = self._param_end(i, b)
                self.drop(i, end + 1 if self.t(end) == "," else end)
                i = end + 1
                first = False
                continue
            first = False
            if self.t(i) == "...":
                i += 1
            name = self.t(i)
            if self.t(i) in ("{", "["):
                i = self.match[i] + 1
            else:
                i += 1
            if mods and ctor:
                props.append(name)
            if self.t(i) == "?":
                self.dropped.add(i)
                i += 1
            if self.t(i) == ":":
                j = self.skip_type(i + 1)
                self.drop(i, j)
                i = j
            end = self._param_end(i, b)
            if self.t(i) == "=":
                self.walk(i + 1, end)
            elif i != end:
                raise EraseError(f"{self.name}: unexpected token in parameter at {self.toks[i].start}: {self.t(i)!r}")
            i = end + 1
            del start
        return props

    def _param_end(self, i: int, b: int) -> int:
        while i < b and self.t(i) != ",":
            if self.t(i) in ("(", "[", "{"):
                i = self.match[i]
            i += 1
        return i

    # ---- function-like: [<T>] (params) [: R] {body} ------------------------------------------
    def func_tail(self, i: int, ctor: bool = False) -> Tuple[int, List[str], int]:
        """i at `<` or `(`. Returns (index after, parameter properties, body-open index or -1)."""
        if self.t(i) == "<":
            j = self.skip_type_args(i)
            self.drop(i, j)
            i = j
        if self.t(i) != "(":
            raise EraseError(f"{self.name}: expected ( at {self.toks[i].start}")
        close = self.match[i]
        props = self.params(i, close, ctor)
        i = close + 1
        if self.t(i) == ":":
            j = self.skip_type(i + 1)
            self.drop(i, j)
            i = j
        if self.t(i) == "{":
            self.walk(i + 1, self.match[i])
            return self.match[i] + 1, props, i
        return i, props, -1

    # ---- generic code walker ---------------------------------------------------------------
    def walk(self, a: int, b: int) -> None:
        i = a
        while i < b:
            i = self.step(i, b)

    def stmt_start(self, i: int) -> bool:
        p = self.t(i - 1)
        return i == 0 or p in (";", "{", "}", "export", "default")

    def step(self, i: int, b: int) -> int:
        tk = self.toks[i]
        x = tk.text
        prev = self.t(i - 1)
        after_dot = prev in (".", "?.")
        if tk.kind == "id" and not after_dot:
            if x == "import" and self.t(i + 1) != "(":
                return self.import_decl(i)
            if x == "export":
                return self.export_decl(i)
            if x == "interface" and self.is_id(i + 1) and self.stmt_start(i):
                j = i + 2
                while self.t(j) != "{":
                    j += 1
                self.drop(i, self.match[j] + 1)
                return self.match[j] + 1
            if x == "type" and self.is_id(i + 1) and self.t(i + 2) in ("=", "<") and self.stmt_start(i):
                j = i + 2
                if self.t(j) == "<":
                    j = self.skip_type_args(j)
                j = self.skip_type(j + 1)
                if self.t(j) == ";":
                    j += 1
                self.drop(i, j)
                return j
            if x == "declare" and self.is_id(i + 1) and self.stmt_start(i):
                j = i
                while self.t(j) != ";":
                    j = self.match[j] if self.t(j) in ("(", "[", "{") else j
                    j += 1
                self.drop(i, j + 1)
                return j + 1
            if x == "enum" or (x == "const" and self.t(i + 1) == "enum"):
                return self.enum_decl(i, i)
            if x == "abstract" and self.t(i + 1) == "class":
                self.dropped.add(i)
                return self.class_decl(i + 1)
            if x == "class" and prev != ".":
                return self.class_decl(i)
            if x == "function":
                j = i + 1
                if self.t(j) == "*":
                    j += 1
                if self.is_id(j):
                    if i == 0 or self.stmt_start(i) or prev == "export" or prev == "default":
                        self.local_values.add(self.t(j)) if self._top(i) else None
                    j += 1
                end, _, body = self.func_tail(j)
                if body < 0:  # overload signature
                    k = end
                    if self.t(k) == ";":
                        k += 1
                    self.drop(i, k)
                    return k
                return end
            if x in ("let", "const", "var"):
                return self.var_decl(i, b)
            if x == "as" and (self.ends_operand(i - 1) or prev == "}"):
                if self.t(i + 1) == "const":
                    self.drop(i, i + 2)
                    return i + 2
                j = self.skip_type(i + 1)
                self.drop(i, j)
                return j
            if self.t(i + 1) == "(" and x not in ("if", "while", "for", "switch", "catch", "with", "function",
                                                  "return", "typeof", "await", "super", "new"):
                close = self.match[i + 1]
                nxt = self.t(close + 1)
                if nxt == "{" or (nxt == ":" and self._colon_then_brace(close + 1)):
                    # method shorthand / accessor in an object literal
                    end, _, body = self.func_tail(i + 1)
                    return end
        if tk.kind == "id" and self.t(i + 1) == "<" and x not in KEYWORDS_BEFORE_EXPR:
            j = self.try_type_args(i + 1)
            if j > 0 and self.t(j) == "(":
                self.drop(i + 1, j)  # explicit type arguments of a call / new
                return j
        if x == "(":
            close = self.match[i]
            nxt = self.t(close + 1)
            if nxt == "=>":
                self.params(i, close)
                return close + 1
            if nxt == ":" and not self._is_ternary_colon(i, close):
                try:
                    j = self.skip_type(close + 2)
                except (EraseError, IndexError):
                    j = -1
                if j > 0 and self.t(j) == "=>":
                    self.params(i, close)
                    self.drop(close + 1, j)
                    return j
            self.walk(i + 1, close)
            return close + 1
        if x in ("[", "{"):
            self.walk(i + 1, self.match[i])
            return self.match[i] + 1
        if x == "<" and not self.ends_operand(i - 1):
            # assertion <T>expr; an asserted object literal keeps parentheses (`=> <T>{...}`)
            j = self.skip_type_args(i)
            self.drop(i, j)
            if self.t(j) == "{":
                self.ins_before.setdefault(j, []).append("(")
                self.ins_after.setdefault(self.match[j], []).append(")")
            return j
        if x == "!" and self.ends_operand(i - 1) and self.t(i + 1) not in ("=", "=="):
            self.dropped.add(i)
            return i + 1
        if x in ("?.", "??"):
            raise EraseError(f"{self.name}: unpatched {x} at {tk.start}")
        return i + 1

    def _top(self, i: int) -> bool:
        depth = 0
        for j in range(i):
            if self.t(j) in ("{", "(", "["):
                depth += 1
            elif self.t(j) in ("}", ")", "]"):
                depth -= 1
        return depth == 0

    def _colon_then_brace(self, i: int) -> bool:
        try:
            j = self.skip_type(i + 1)
        except (EraseError, IndexError):
            return False
        return self.t(j) == "{"

    def _is_ternary_colon(self, a: int, close: int) -> bool:
        """`(x) :` is a ternary branch when a `?` precedes at the same nesting level."""
        depth = 0
        j = a - 1
        while j >= 0:
            x = self.t(j)
            if x in (")", "]", "}"):
                j = self.match[j]
            elif x in ("(", "[", "{", ";", ","):
                return False
            elif x == "?":
                return True
            elif x == ":" or x == "=>":
                return False
            j -= 1
        return False

    # ---- declarations ----------------------------------------------------------------------
    def var_decl(self, i: int, b: int) -> int:
        top = self._top(i)
        j = i + 1
        while True:
            if self.t(j) in ("{", "["):
                j = self.match[j] + 1
            else:
                if top:
                    self.local_values.add(self.t(j))
                j += 1
            if self.t(j) == "!":
                self.dropped.add(j)
                j += 1
            if self.t(j) == ":":
                k = self.skip_type(j + 1)
                self.drop(j, k)
                j = k
            if self.t(j) == "=":
                k = j + 1
                while k < b and self.t(k) not in (",", ";") and not (self.t(k) in ("of", "in") and False):
                    if self.t(k) in (")", "]", "}"):
                        break
                    k = self.step(k, b)
                j = k
            if self.t(j) == ",":
                j += 1
                continue
            return j

    def enum_decl(self, i: int, stmt: int) -> int:
        j = i
        if self.t(j) == "const":
            j += 1
        name = self.t(j + 1)
        open_ = j + 2
        close = self.match[open_]
        members = []
        k = open_ + 1
        while k < close:
            mname = self.t(k)
            if self.toks[k].kind == "str":
                mname = mname[1:-1]
            k += 1
            init = None
            if self.t(k) == "=":
                e = k + 1
                while e < close and self.t(e) != ",":
                    e = self.match[e] + 1 if self.t(e) in ("(", "[", "{") else e + 1
                init = self.src[self.toks[k + 1].start:self.toks[e - 1].end]
                k = e
            if self.t(k) == ",":
                k += 1
            members.append((mname, init))
        lines = [f"var {name} = (function () {{ const E = {{}};"]
        prevn = None
        for mname, init in members:
            val = init if init is not None else ("0" if prevn is None else f"{prevn} + 1")
            lines.append(f" const {mname} = {val}; E[{mname!r}] = {mname}; if (typeof {mname} === \"number\") E[{mname}] = {mname!r};")
            prevn = mname
        lines.append(" return E; })();")
        self.drop(i, close + 1)
        self.ins_before.setdefault(i, []).append("".join(lines))
        self.local_values.add(name)
        return close + 1

    def class_decl(self, i: int) -> int:
        j = i + 1
        name = None
        if self.is_id(j) and self.t(j) not in ("extends", "implements"):
            name = self.t(j)
            if self._top(i):
                self.local_values.add(name)
            j += 1
        if self.t(j) == "<":
            k = self.skip_type_args(j)
            self.drop(j, k)
            j = k
        derived = False
        if self.t(j) == "extends":
            derived = True
            j += 1
            while self.t(j) not in ("{", "implements"):
                if self.t(j) == "<":
                    k = self.skip_type_args(j)
                    self.drop(j, k)
                    j = k
                    continue
                j = self.step(j, self.n)
        if self.t(j) == "implements":
            k = j
            while self.t(k) != "{":
                k = self.match[k] + 1 if self.t(k) in ("(", "[") else k + 1
            self.drop(j, k)
            j = k
        assert self.t(j) == "{", (self.name, self.toks[j].start)
        close = self.match[j]
        self.class_body(j, close, derived)
        return close + 1

    def class_body(self, a: int, b: int, derived: bool) -> None:
        i = a + 1
        inits: List[str] = []
        ctor: Optional[Tuple[int, List[str]]] = None
        while i < b:
            if self.t(i) == ";":
                i += 1
                continue
            start = i
            mods: List[str] = []
            while self.t(i) in MEMBER_MODIFIERS and self.t(i + 1) not in ("(", ":", "=", ";", "?", "!", "<", "}"):
                mods.append(self.t(i))
                if self.t(i) in TS_ONLY_MODIFIERS:
                    self.dropped.add(i)
                i += 1
            if self.t(i) == "[" and self.is_id(i + 1) and self.t(i + 2) == ":":  # index signature
                e = self._member_end(i)
                self.drop(start, e)
                i = e
                continue
            name_i = i
            name = self.t(i)
            if self.t(i) == "[":
                self.walk(i + 1, self.match[i])
                i = self.match[i] + 1
            else:
                i += 1
            if self.t(i) in ("?", "!"):
                self.dropped.add(i)
                i += 1
            if self.t(i) in ("(", "<"):
                end, props, body = self.func_tail(i, ctor=name == "constructor")
                if body < 0 or "abstract" in mods or "declare" in mods:
                    if self.t(end) == ";":
                        end += 1
                    self.drop(start, end)
                elif name == "constructor":
                    ctor = (body, props)
                i = end
                continue
            # property
            if self.t(i) == ":":
                k = self.skip_type(i + 1)
                self.drop(i, k)
                i = k
            if "abstract" in mods or "declare" in mods:
                e = self._member_end(i)
                self.drop(start, e)
                i = e
                continue
            if self.t(i) == "=":
                e = self._member_end(i)
                init_end = e - 1 if self.t(e - 1) == ";" else e
                self.walk(i + 1, init_end)
                if "static" in mods:
                    i = e
                    continue
                expr = self.render(i + 1, init_end).strip()
                self.extra_uses.update(self.toks[k].text for k in range(i + 1, init_end)
                                       if k not in self.dropped and self.toks[k].kind == "id")
                key = f"[{self.render(name_i + 1, self.match[name_i]).strip()}]" if name == "[" else (
                    f"[{name}]" if self.toks[name_i].kind == "str" else f".{name}")
                inits.append(f"this{key} = {expr};")
                self.drop(start, e)
                i = e
                continue
            if self.t(i) == ";":
                self.drop(start, i + 1)
                i += 1
                continue
            raise EraseError(f"{self.name}: cannot parse class member at {self.toks[start].start}: {self.t(start)!r}")
        if ctor is not None:
            body, props = ctor
            assigns = [f"this.{p} = {p};" for p in props] + inits
            if assigns:
                at = self._after_super(body) if derived else body
                self.ins_after.setdefault(at, []).append(" " + " ".join(assigns))
        elif inits:
            sup = "constructor(...args) { super(...args); " if derived else "constructor() { "
            self.ins_after.setdefault(a, []).append(" " + sup + " ".join(inits) + " }")

    def _after_super(self, body: int) -> int:
        """Token index after which parameter properties / initializers go: after `super(...);`."""
        close = self.match[body]
        i = body + 1
        while i < close:
            if self.t(i) == "super" and self.t(i + 1) == "(":
                j = self.match[i + 1] + 1
                return j if self.t(j) == ";" else j - 1
            if self.t(i) in ("(", "[", "{"):
                i = self.match[i]
            i += 1
        return body

    def _member_end(self, i: int) -> int:
        while self.t(i) != ";":
            if self.t(i) in ("(", "[", "{"):
                i = self.match[i]
            i += 1
        return i + 1

    # ---- modules -----------------------------------------------------------------------------
    def import_decl(self, i: int) -> int:
        j = i + 1
        if self.t(j) == "type" and self.t(j + 1) != "from":  # import type {...}
            e = self._stmt_end(j)
            self.drop(i, e)
            return e
        default = ns = None
        named: List[Tuple[str, str]] = []
        if self.toks[j].kind == "str":
            spec = self.t(j)[1:-1]
            e = self._stmt_end(j)
            self.imports.append((spec, None, None, [], (i, e)))
            return e
        if self.is_id(j) and self.t(j) != "from":
            default = self.t(j)
            j += 1
            if self.t(j) == ",":
                j += 1
        if self.t(j) == "*":
            ns = self.t(j + 2)
            j += 3
        if self.t(j) == "{":
            close = self.match[j]
            k = j + 1
            while k < close:
                orig = self.t(k)
                local = orig
                if self.t(k + 1) == "as":
                    local = self.t(k + 2)
                    k += 2
                named.append((orig, local))
                k += 1
                if self.t(k) == ",":
                    k += 1
            j = close + 1
        assert self.t(j) == "from", (self.name, self.toks[j].start)
        spec = self.t(j + 1)[1:-1]
        e = self._stmt_end(j + 1)
        self.imports.append((spec, default, ns, named, (i, e)))
        return e

    def value_uses(self) -> Set[str]:
        """Identifiers still referenced as values after erasure (TypeScript elides an import whose
        bindings are used only in type positions, which also decides module evaluation order)."""
        used = set(self.extra_uses)
        for k, tk in enumerate(self.toks):
            if tk.kind == "id" and k not in self.dropped and self.t(k - 1) not in (".", "?."):
                used.add(tk.text)
        return used

    def _stmt_end(self, j: int) -> int:
        while self.t(j) != ";" and j < self.n:
            j += 1
        return j + 1

    def export_decl(self, i: int) -> int:
        j = i + 1
        x = self.t(j)
        if x == "*":
            spec = self.t(j + 2)[1:-1]
            e = self._stmt_end(j)
            self.star_from.append(spec)
            self.reexports.append((spec, [("*", "*")], (i, e)))
            return e
        if x == "{":
            close = self.match[j]
            names = []
            k = j + 1
            while k < close:
                orig = self.t(k)
                alias = orig
                if self.t(k + 1) == "as":
                    alias = self.t(k + 2)
                    k += 2
                names.append((orig, alias))
                k += 1
                if self.t(k) == ",":
                    k += 1
            if self.t(close + 1) == "from":
                spec = self.t(close + 2)[1:-1]
                e = self._stmt_end(close + 2)
                self.reexports.append((spec, names, (i, e)))
                return e
            e = self._stmt_end(close)
            self.local_exports.append((names, (i, e)))
            return e
        if x in ("interface", "type") or (x == "declare"):
            k = self.step(j, self.n)
            self.dropped.add(i)
            return k
        if x == "default":
            return j + 1
        # export class / function / const / enum / abstract class
        before = set(self.local_values)
        k = self.step(j, self.n)
        for nm in self.local_values - before:
            self.exports.add(nm)
        if x in ("enum",) or (x == "const" and self.t(j + 1) == "enum"):
            pass
        return k


# ---- project ------------------------------------------------------------------------------
PATCHES = {
    # optional chaining / nullish coalescing (Node 12 has neither); exact textual lowering
    "client.ts": [
        ("return this.mergeTree.pendingSegments?.last();",
         "return this.mergeTree.pendingSegments == null ? undefined : this.mergeTree.pendingSegments.last();"),
        ("return this.mergeTree.pendingSegments?.some(",
         "return this.mergeTree.pendingSegments == null ? undefined : this.mergeTree.pendingSegments.some("),
        ("if (this.mergeTree.options?.newMergeTreeSnapshotFormat === true) {",
         "if ((this.mergeTree.options == null ? undefined : this.mergeTree.options.newMergeTreeSnapshotFormat) === true) {"),
    ],
    "snapshotChunks.ts": [
        ("headerMetadata?.totalLength,", "(headerMetadata == null ? undefined : headerMetadata.totalLength),"),
        ("headerMetadata?.totalSegmentCount,", "(headerMetadata == null ? undefined : headerMetadata.totalSegmentCount),"),
        ("headerMetadata?.sequenceNumber,", "(headerMetadata == null ? undefined : headerMetadata.sequenceNumber),"),
        ("headerMetadata?.minSequenceNumber,", "(headerMetadata == null ? undefined : headerMetadata.minSequenceNumber),"),
    ],
    "snapshotLoader.ts": [
        ('this.runtime.clientId ?? "snapshot",', '(this.runtime.clientId != null ? this.runtime.clientId : "snapshot"),'),
    ],
    "snapshotV1.ts": [
        ("this.chunkSize = mergeTree?.options?.mergeTreeSnapshotChunkSize ?? SnapshotV1.chunkSize;",
         "this.chunkSize = __nc(mergeTree == null || mergeTree.options == null ? undefined : "
         "mergeTree.options.mergeTreeSnapshotChunkSize, SnapshotV1.chunkSize);"),
    ],
    "snapshotlegacy.ts": [
        ("this.chunkSize = mergeTree?.options?.mergeTreeSnapshotChunkSize ?? SnapshotLegacy.sizeOfFirstChunk;",
         "this.chunkSize = __nc(mergeTree == null || mergeTree.options == null ? undefined : "
         "mergeTree.options.mergeTreeSnapshotChunkSize, SnapshotLegacy.sizeOfFirstChunk);"),
        ("path: this.mergeTree.options?.catchUpBlobName ?? SnapshotLegacy.catchupOps,",
         "path: __nc(this.mergeTree.options == null ? undefined : this.mergeTree.options.catchUpBlobName, "
         "SnapshotLegacy.catchupOps),"),
    ],
}
NC_HELPER = "const __nc = (a, b) => (a !== null && a !== undefined ? a : b);\n"


def apply_patches(name: str, src: str) -> str:
    for old, new in PATCHES.get(name, []):
        if src.count(old) != 1:
            raise EraseError(f"{name}: patch target not found exactly once: {old}")
        src = src.replace(old, new)
    if name in PATCHES and "__nc(" in src:
        src = NC_HELPER + src
    return src


SHIMS = {
    "@fluidframework/common-utils": ("_shim_common_utils", {"Trace", "fromBase64ToUtf8", "IsoBuffer", "assert"}),
    "@fluidframework/protocol-definitions": ("_shim_protocol", {"MessageType", "FileMode", "TreeEntry"}),
    "@fluidframework/container-definitions": ("_shim_container", {"AttachState"}),
    "@fluidframework/telemetry-utils": ("_shim_telemetry", {"ChildLogger"}),
    # type-only packages: every named import from them is erased
    "@fluidframework/core-interfaces": ("_shim_types", set()),
    "@fluidframework/datastore-definitions": ("_shim_types", set()),
    "@fluidframework/common-definitions": ("_shim_types", set()),
    "@fluidframework/runtime-definitions": ("_shim_types", set()),
}
SHIM_SRC = {
    "_shim_common_utils": """// shim of @fluidframework/common-utils (trace.ts:12-33, base64Encoding, IsoBuffer) for the oracle run
export class Trace {
    static start() { return new Trace(Date.now()); }
    constructor(start) { this.startTick = start; this.lastTick = start; }
    trace() { const now = Date.now(); const e = { totalTimeElapsed: now - this.startTick, duration: now - this.lastTick, tick: now }; this.lastTick = now; return e; }
}
export const fromBase64ToUtf8 = (s) => Buffer.from(s, "base64").toString("utf8");
export const IsoBuffer = Buffer;
export function assert(c, m) { if (!c) throw new Error(m || "assert"); }
""",
    "_shim_protocol": """// shim of @fluidframework/protocol-definitions (protocol.ts:6-32, storage.ts:28, 73)
export const MessageType = { Operation: "op", NoOp: "noop" };
export const FileMode = { File: "100644", Directory: "040000", Executable: "100755", Symlink: "120000" };
export const TreeEntry = { Blob: "Blob", Commit: "Commit", Tree: "Tree", Attachment: "Attachment" };
""",
    "_shim_container": """// shim of @fluidframework/container-definitions (runtime.ts:33)
export const AttachState = { Detached: "Detached", Attaching: "Attaching", Attached: "Attached" };
""",
    "_shim_types": "// type-only packages have no runtime exports\nexport {};\n",
    "_shim_telemetry": """// shim of @fluidframework/telemetry-utils: a logger that records nothing
// TelemetryLogger.shipAssert reports a failed condition as an error event; it does not throw
const nop = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {}, shipAssert() {} };
export const ChildLogger = { create() { return nop; } };
""",
}


def resolve(spec: str, files: Set[str]) -> Tuple[str, Optional[Set[str]]]:
    """module specifier -> (output module name, its runtime exports if known statically)."""
    if spec in SHIMS:
        name, exports = SHIMS[spec]
        return "./" + name + ".mjs", exports
    if spec.startswith("."):
        base = spec[2:] if spec.startswith("./") else spec
        if base in ("", "index"):
            base = "index"
        if base not in files:
            raise EraseError(f"unknown module {spec}")
        return "./" + base + ".mjs", None
    if spec in ("assert",):
        return spec, None
    raise EraseError(f"no shim for {spec}")


def erase_project(src_dir: str, out_dir: str, names: List[str], extra: Optional[Dict[str, str]] = None) -> None:
    mods: Dict[str, Module] = {}
    sources = []
    for nm in names:
        with open(os.path.join(src_dir, nm + ".ts")) as f:
            sources.append((nm, apply_patches(nm + ".ts", f.read())))
    sources.extend((extra or {}).items())
    for nm, src in sources:
        m = Module(nm, src)
        m.walk(0, m.n)
        mods[nm] = m
    files = set(mods)
    # runtime exports: direct declarations + local `export {}` + re-exports (fixpoint)
    exp: Dict[str, Set[str]] = {}
    imported_values: Dict[str, Set[str]] = {nm: set() for nm in mods}
    for nm, m in mods.items():
        exp[nm] = set(m.exports)
    changed = True
    while changed:
        changed = False
        for nm, m in mods.items():
            # runtime-valued imports (needed to decide `export { X }` of an imported name)
            vals = set()
            for spec, default, ns, named, _ in m.imports:
                target, known = resolve(spec, files)
                tset = known if known is not None else (exp.get(target[2:-4]) if target.startswith("./") else None)
                for orig, local in named:
                    if tset is None or orig in tset:
                        vals.add(local)
                if default:
                    vals.add(default)
                if ns:
                    vals.add(ns)
            imported_values[nm] = vals
            new = set(exp[nm])
            for names_, _ in m.local_exports:
                for orig, alias in names_:
                    if orig in m.local_values or orig in vals:
                        new.add(alias)
            for spec, names_, _ in m.reexports:
                target, known = resolve(spec, files)
                tset = known if known is not None else exp.get(target[2:-4], set())
                for orig, alias in names_:
                    if orig == "*":
                        new |= tset
                    elif orig in tset:
                        new.add(alias)
            if new != exp[nm]:
                exp[nm] = new
                changed = True
    os.makedirs(out_dir, exist_ok=True)
    for nm, m in mods.items():
        for spec, default, ns, named, (a, b) in m.imports:
            m.drop(a, b)  # import statements are not value uses of their own bindings
        used = m.value_uses()
        for names_, _ in m.local_exports:
            used.update(o for o, _ in names_)
        for spec, default, ns, named, (a, b) in m.imports:
            target, known = resolve(spec, files)
            tset = known if known is not None else (exp[target[2:-4]] if target.startswith("./") else None)
            keep = [(o, l) for o, l in named if (tset is None or o in tset) and l in used]
            parts = []
            if default and default in used:
                parts.append(default)
            if ns and ns in used:
                parts.append(f"* as {ns}")
            if keep:
                parts.append("{ " + ", ".join(o if o == l else f"{o} as {l}" for o, l in keep) + " }")
            m.drop(a, b)
            if parts:
                m.ins_before.setdefault(a, []).append(f'import {", ".join(parts)} from "{target}";')
            elif not named and default is None and ns is None:
                m.ins_before.setdefault(a, []).append(f'import "{target}";')
        for names_, (a, b) in m.local_exports:
            keep = [(o, al) for o, al in names_ if o in m.local_values or o in imported_values[nm]]
            m.drop(a, b)
            if keep:
                m.ins_before.setdefault(a, []).append(
                    "export { " + ", ".join(o if o == al else f"{o} as {al}" for o, al in keep) + " };")
        for spec, names_, (a, b) in m.reexports:
            target, known = resolve(spec, files)
            tset = known if known is not None else exp[target[2:-4]]
            m.drop(a, b)
            if names_ == [("*", "*")]:
                m.ins_before.setdefault(a, []).append(f'export * from "{target}";')
                continue
            keep = [(o, al) for o, al in names_ if o in tset]
            if keep:
                m.ins_before.setdefault(a, []).append(
                    "export { " + ", ".join(o if o == al else f"{o} as {al}" for o, al in keep) + f' }} from "{target}";')
        with open(os.path.join(out_dir, nm + ".mjs"), "w") as f:
            f.write(m.render())
    for nm, src in SHIM_SRC.items():
        with open(os.path.join(out_dir, nm + ".mjs"), "w") as f:
            f.write(src)


MT_FILES = ["base", "client", "collections", "constants", "index", "localReference", "mergeTree",
            "mergeTreeDeltaCallback", "mergeTreeTracking", "opBuilder", "ops", "partialLengths", "properties",
            "segmentGroupCollection", "segmentPropertiesManager", "snapshotChunks", "snapshotLoader", "snapshotV1",
            "snapshotlegacy", "sortedSegmentSet", "textSegment", "text"]


MATRIX_SRC = "/root/reference/packages/dds/matrix/src"


def matrix_sources(matrix_dir: str) -> Dict[str, str]:
    """SharedMatrix's PermutationSegment (permutationvector.ts:36-122) and the Handle constants it
    uses (handletable.ts), as two extra modules over the erased merge-tree. Only the segment class is
    taken: PermutationVector itself needs the runtime (and asserts on annotate deltas,
    permutationvector.ts:337), while config 5 replays raw Client ops on PermutationSegment rows."""
    with open(os.path.join(matrix_dir, "handletable.ts")) as f:
        handletable = f.read()
    with open(os.path.join(matrix_dir, "permutationvector.ts")) as f:
        pv = f.read()
    m = Module("permutationvector", pv)
    k = next(i for i, t in enumerate(m.toks) if t.text == "class" and m.t(i + 1) == "PermutationSegment")
    j = k
    while m.t(j) != "{":
        j += 1
    cls = pv[m.toks[k - 1].start:m.toks[m.match[j]].end]
    head = ('import { strict as assert } from "assert";\n'
            'import { BaseSegment, LocalReferenceCollection } from "./index";\n'
            'import { Handle, isHandleValid } from "./handletable";\n')
    old = "this.next = (this.handles[free] as Handle) ?? (free + 1);"
    if handletable.count(old) != 1:
        raise EraseError("handletable.ts: patch target not found")
    handletable = NC_HELPER + handletable.replace(old, "this.next = __nc(this.handles[free] as Handle, free + 1);")
    return {"handletable": handletable, "permutationSegment": head + cls + "\n"}


SEQUENCE_SRC = "/root/reference/packages/dds/sequence/src"


def sequence_sources(seq_dir: str) -> Dict[str, str]:
    """The sequence package's SubSequence segment (sharedSequence.ts:12-101: SharedObjectSequence / SharedNumberSequence
    items) and its MaxRun constant, as one extra module over the erased merge-tree. Only the segment class is taken:
    SharedSequence itself needs the container runtime, while the fixtures replay raw Client ops on SubSequence rows."""
    with open(os.path.join(seq_dir, "sharedSequence.ts")) as f:
        src = f.read()
    m = Module("sharedSequence", src)
    k = next(i for i, t in enumerate(m.toks) if t.text == "class" and m.t(i + 1) == "SubSequence")
    j = k
    while m.t(j) != "{":
        j += 1
    cls = src[m.toks[k - 1].start:m.toks[m.match[j]].end]
    c = next(i for i, t in enumerate(m.toks) if t.text == "const" and m.t(i + 1) == "MaxRun")
    e = c
    while m.t(e) != ";":
        e += 1
    maxrun = src[m.toks[c].start:m.toks[e].end]
    head = 'import { BaseSegment, LocalReferenceCollection } from "./index";\n'
    return {"subSequence": head + maxrun + "\n" + cls + "\n"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default="/root/reference/packages/dds/merge-tree/src")
    ap.add_argument("--out", default="/tmp/mt-oracle")
    ap.add_argument("--matrix", default=MATRIX_SRC)
    ap.add_argument("--sequence", default=SEQUENCE_SRC)
    args = ap.parse_args()
    if os.path.abspath(args.out).startswith(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))):
        raise SystemExit("the erased reference must not be written inside the repository")
    erase_project(args.src, args.out, MT_FILES, {**matrix_sources(args.matrix), **sequence_sources(args.sequence)})
    print(f"erased {len(MT_FILES)} merge-tree modules + PermutationSegment + SubSequence into {args.out}")


if __name__ == "__main__":
    sys.exit(main())
