"""A minimal Clojure reader for static checks of the JVM glue (no JDK in the
image): strings, comments, character literals, ( ) [ ] { } #{ } forms,
quote/deref/syntax-quote prefixes, ^metadata (dropped). Raises ValueError on
unbalanced input. Test infrastructure only."""
from __future__ import annotations

from typing import List


class Form(list):
    """A bracketed form; .kind is '(' '[' '{' or '#{'; .line its first line."""
    kind = "("
    line = 0


class Str(str):
    """A string literal (kept apart from symbols)."""


_CLOSE = {"(": ")", "[": "]", "{": "}", "#{": "}"}
_DELIM = " \t\r\n,()[]{}\";"


class _Reader:
    def __init__(self, text: str):
        self.t, self.i, self.n, self.line = text, 0, len(text), 1

    def _skip_ws(self):
        t = self.t
        while self.i < self.n:
            c = t[self.i]
            if c == "\n":
                self.line += 1
                self.i += 1
            elif c in " \t\r,":
                self.i += 1
            elif c == ";":
                while self.i < self.n and t[self.i] != "\n":
                    self.i += 1
            else:
                return

    def read(self, closer=None):
        """Next form; None at the end of input or at `closer`."""
        self._skip_ws()
        if self.i >= self.n:
            if closer:
                raise ValueError(f"missing {closer!r} at end of input")
            return None
        t, c = self.t, self.t[self.i]
        if c in ")]}":
            if c != closer:
                raise ValueError(f"unbalanced {c!r} at line {self.line}")
            self.i += 1
            return None
        if c == '"':
            j, buf = self.i + 1, []
            while j < self.n and t[j] != '"':
                if t[j] == "\\":
                    buf.append(t[j:j + 2])
                    j += 2
                    continue
                if t[j] == "\n":
                    self.line += 1
                buf.append(t[j])
                j += 1
            if j >= self.n:
                raise ValueError(f"unterminated string at line {self.line}")
            self.i = j + 1
            return Str("".join(buf))
        if c == "\\":  # character literal
            j = self.i + 2
            while j < self.n and t[j].isalnum():
                j += 1
            s, self.i = t[self.i:j], j
            return s
        if c in "([{" or t.startswith("#{", self.i):
            kind = "#{" if t.startswith("#{", self.i) else c
            f = Form()
            f.kind, f.line = kind, self.line
            self.i += len(kind)
            while True:
                x = self.read(_CLOSE[kind])
                if x is None:
                    return f
                f.append(x)
        if c == "^":  # metadata: drop it, return the form it annotates
            self.i += 1
            if self.read() is None:
                raise ValueError(f"dangling ^ at line {self.line}")
            return self.read(closer)
        if c in "'@`~" or t.startswith("#'", self.i) or t.startswith("#(", self.i):
            self.i += 1 if c != "#" else 1
            return self.read(closer)
        j = self.i
        while j < self.n and t[j] not in _DELIM:
            j += 1
        s, self.i = t[self.i:j], j
        return s


def read_all(text: str) -> List[object]:
    r, out = _Reader(text), []
    while True:
        x = r.read()
        if x is None:
            if r.i < r.n:
                raise ValueError(f"unbalanced input at line {r.line}")
            return out
        out.append(x)


def defn_arities(forms) -> dict:
    """name -> (public, [arity, ...]) of every top-level defn/defn-; an arity
    is the count of parameters, -(k+1) when variadic after k."""
    out = {}
    for f in forms:
        if not (isinstance(f, Form) and f.kind == "(" and f and f[0] in ("defn", "defn-")):
            continue
        rest = [x for x in f[2:] if not isinstance(x, Str)]
        rest = [x for x in rest if not (isinstance(x, Form) and x.kind == "{")]  # attr-map
        if rest and isinstance(rest[0], Form) and rest[0].kind == "[":
            vecs = [rest[0]]
        else:
            vecs = [x[0] for x in rest if isinstance(x, Form) and x.kind == "(" and x and
                    isinstance(x[0], Form) and x[0].kind == "["]
        ar = [-(list(v).index("&") + 1) if "&" in v else len(v) for v in vecs]
        out[f[1]] = (f[0] == "defn", ar)
    return out


def accepts(arities, n: int) -> bool:
    return any(a == n or (a < 0 and n >= -a - 1) for a in arities)


def walk(form):
    yield form
    if isinstance(form, list):
        for x in form:
            yield from walk(x)
