"""Resolve compile-time A/B switches out of the kernel sources: every
#if / #ifndef / #elif / #else / #endif whose condition names only the given macros is evaluated with
their values and dropped, keeping the chosen branch; `#ifndef NAME` default-definition blocks of those
macros go too.  Other conditionals are left alone.  usage:
  python tools/unifdef_switches.py NAME=VALUE [NAME=VALUE ...] -- file [file ...]"""
import re
import sys


def main(argv):
    sep = argv.index("--")
    vals = dict(a.split("=", 1) for a in argv[:sep])
    files = argv[sep + 1:]
    ident = re.compile(r"[A-Za-z_][A-Za-z0-9_]*")

    def cond_value(expr):
        names = set(ident.findall(expr)) - {"defined"}
        if not names or not names <= set(vals):
            return None
        e = expr
        for n in sorted(names, key=len, reverse=True):
            e = re.sub(r"\b%s\b" % n, vals[n].rstrip("uU"), e)
        e = e.replace("&&", " and ").replace("||", " or ").replace("!", " not ").replace(" not =", "!=")
        return bool(eval(e))

    for path in files:
        out, stack = [], []  # frame: [kind, taking, taken]  kind 'keep' | 'eval'
        for line in open(path).read().split("\n"):
            s = line.strip()
            m = re.match(r"#\s*(ifndef|ifdef|if|elif|else|endif)\b(.*)", s)
            live = all(f[1] for f in stack if f[0] == "eval")
            if m:
                d, rest = m.group(1), m.group(2).split("//")[0].strip()
                if d in ("if", "ifdef", "ifndef"):
                    v = None
                    if d == "if":
                        v = cond_value(rest)
                    elif rest in vals:
                        v = (d == "ifdef")  # a resolved switch counts as defined: its default block goes
                    if v is None:
                        stack.append(["keep", True, True])
                        if live:
                            out.append(line)
                    else:
                        stack.append(["eval", v, v])
                    continue
                f = stack[-1]
                if f[0] == "keep":
                    if d == "endif":
                        stack.pop()
                    if all(g[1] for g in stack if g[0] == "eval"):
                        out.append(line)
                    continue
                if d == "elif":
                    v = cond_value(rest)
                    assert v is not None, (path, line)
                    f[1] = (not f[2]) and v
                    f[2] = f[2] or v
                elif d == "else":
                    f[1] = not f[2]
                    f[2] = True
                else:
                    stack.pop()
                continue
            if live:
                out.append(line)
        assert not stack, path
        open(path, "w").write("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1:])
