"""A small parser for R function definitions `name <- function(formals) body` at top level:
name -> [(argument, default source text or None)].  Comments and string literals are honoured;
defaults are compared after removing whitespace.  TEST INFRASTRUCTURE (tests/test_r_surface.py,
tests/golden/make_r_formals.py)."""
import re

_DEF = re.compile(r"^([A-Za-z._][A-Za-z0-9._]*)\s*(?:<-|=)\s*function\s*\(", re.M)


def _strip_comments(src: str) -> str:
    out, i, n = [], 0, len(src)
    quote = None
    while i < n:
        ch = src[i]
        if quote:
            out.append(ch)
            if ch == "\\" and i + 1 < n:
                out.append(src[i + 1])
                i += 2
                continue
            if ch == quote:
                quote = None
        elif ch in "\"'`":
            quote = ch
            out.append(ch)
        elif ch == "#":
            while i < n and src[i] != "\n":
                i += 1
            continue
        else:
            out.append(ch)
        i += 1
    return "".join(out)


def _split_top(s: str):
    parts, depth, cur, quote = [], 0, [], None
    i = 0
    while i < len(s):
        ch = s[i]
        if quote:
            cur.append(ch)
            if ch == "\\" and i + 1 < len(s):
                cur.append(s[i + 1])
                i += 2
                continue
            if ch == quote:
                quote = None
        elif ch in "\"'`":
            quote = ch
            cur.append(ch)
        elif ch in "([{":
            depth += 1
            cur.append(ch)
        elif ch in ")]}":
            depth -= 1
            cur.append(ch)
        elif ch == "," and depth == 0:
            parts.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
        i += 1
    if "".join(cur).strip():
        parts.append("".join(cur))
    return parts


def _norm(expr: str) -> str:
    return re.sub(r"\s+", "", expr)


def parse_formals(src: str) -> dict:
    """{name: [(arg, default-or-None), ...]} for every top-level `name <- function(...)`; a name
    defined twice keeps its last definition (as sourcing the file would)."""
    src = _strip_comments(src)
    out = {}
    for m in _DEF.finditer(src):
        i, depth, quote = m.end(), 1, None
        start = i
        while depth:
            ch = src[i]
            if quote:
                if ch == "\\":
                    i += 1
                elif ch == quote:
                    quote = None
            elif ch in "\"'`":
                quote = ch
            elif ch == "(":
                depth += 1
            elif ch == ")":
                depth -= 1
            i += 1
        args = []
        for part in _split_top(src[start:i - 1]):
            if "=" in part and not re.match(r"^\s*[A-Za-z._][A-Za-z0-9._]*\s*$", part):
                k, v = part.split("=", 1)
                args.append((k.strip(), _norm(v)))
            else:
                args.append((part.strip(), None))
        out[m.group(1)] = args
    return out
