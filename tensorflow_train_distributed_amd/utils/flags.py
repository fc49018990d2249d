"""gflags-style command-line flags (the `tf.app.flags` surface the reference uses).

Reference: `tf.app.flags.DEFINE_string/DEFINE_integer/DEFINE_boolean` + `FLAGS`
(/root/reference/distribute_training.py:22-36) and `tf.app.run()` (:241-242).
Accepted syntaxes: `--name=value`, `--name value`, `--flag`/`--noflag` for booleans.
Flags are parsed lazily on first attribute access (or explicitly by app.run()).
"""
from __future__ import annotations

import sys
from typing import Any, Callable, Dict, List, Optional


class FlagError(ValueError):
    pass


class _Flag:
    __slots__ = ("name", "default", "help", "parser", "value", "present", "is_bool")

    def __init__(self, name, default, help_, parser, is_bool=False):
        self.name = name
        self.default = default
        self.help = help_
        self.parser = parser
        self.value = default
        self.present = False
        self.is_bool = is_bool


def _parse_bool(v):
    if isinstance(v, bool):
        return v
    s = str(v).strip().lower()
    if s in ("1", "true", "t", "yes", "y"):
        return True
    if s in ("0", "false", "f", "no", "n"):
        return False
    raise FlagError("not a boolean: %r" % v)


class FlagValues:
    def __init__(self):
        object.__setattr__(self, "_flags", {})
        object.__setattr__(self, "_parsed", False)

    def _define(self, name, default, help_, parser, is_bool=False):
        if name in self._flags:
            raise FlagError("flag --%s defined twice" % name)
        self._flags[name] = _Flag(name, None if default is None else parser(default), help_, parser, is_bool)

    def __call__(self, argv: List[str]) -> List[str]:
        """Parse argv (argv[0] is the program); returns the unparsed remainder."""
        rest = [argv[0]] if argv else []
        i = 1
        while i < len(argv):
            a = argv[i]
            if a == "--":
                rest.extend(argv[i + 1:])
                break
            if not a.startswith("-") or a == "-":
                rest.append(a)
                i += 1
                continue
            body = a.lstrip("-")
            if "=" in body:
                name, val = body.split("=", 1)
            else:
                name, val = body, None
            fl = self._flags.get(name)
            if fl is None and name.startswith("no") and name[2:] in self._flags and self._flags[name[2:]].is_bool:
                fl, val = self._flags[name[2:]], "false"
            if fl is None:
                rest.append(a)
                i += 1
                continue
            if val is None:
                if fl.is_bool:
                    val = "true"
                elif i + 1 < len(argv):
                    i += 1
                    val = argv[i]
                else:
                    raise FlagError("flag --%s needs a value" % name)
            fl.value = fl.parser(val)
            fl.present = True
            i += 1
        object.__setattr__(self, "_parsed", True)
        return rest

    def __getattr__(self, name):
        flags = object.__getattribute__(self, "_flags")
        if name not in flags:
            raise AttributeError("unknown flag --%s" % name)
        if not object.__getattribute__(self, "_parsed"):
            self(list(sys.argv))
        return flags[name].value

    def __setattr__(self, name, value):
        if name not in self._flags:
            raise AttributeError("unknown flag --%s" % name)
        self._flags[name].value = value

    def __contains__(self, name):
        return name in self._flags

    def flag_values_dict(self) -> Dict[str, Any]:
        return {k: f.value for k, f in self._flags.items()}

    def reset(self):
        for f in self._flags.values():
            f.value = f.default
            f.present = False
        object.__setattr__(self, "_parsed", False)

    def help_text(self):
        return "\n".join("  --%s: %s (default: %r)" % (k, f.help, f.default) for k, f in sorted(self._flags.items()))


FLAGS = FlagValues()


def DEFINE_string(name, default, help_, flag_values=FLAGS):
    flag_values._define(name, default, help_, str)


def DEFINE_integer(name, default, help_, flag_values=FLAGS):
    flag_values._define(name, default, help_, int)


def DEFINE_float(name, default, help_, flag_values=FLAGS):
    flag_values._define(name, default, help_, float)


def DEFINE_boolean(name, default, help_, flag_values=FLAGS):
    flag_values._define(name, default, help_, _parse_bool, is_bool=True)


DEFINE_bool = DEFINE_boolean


def DEFINE_list(name, default, help_, flag_values=FLAGS):
    flag_values._define(name, default, help_, lambda v: v if isinstance(v, list) else [s for s in str(v).split(",") if s])
