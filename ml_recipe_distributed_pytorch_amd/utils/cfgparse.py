"""Dependency-free, configargparse-compatible argument parser.

The reference builds every CLI with ``configargparse`` (``modules/model/utils/parser.py:1-207``):
two parsers (trainer+model or predictor+model) read the *same* argv and the *same* ``-c`` file,
``parse_known_args`` on each, and ``get_params`` aborts only on arguments unknown to *all*
parsers (``parser.py:9-31``).  ``configargparse`` is not installed in this environment, so this
module re-implements the subset of its semantics the recipe relies on:

* ``add_argument(..., is_config_file=True)`` marks an option whose value is a config-file path.
* Config files hold ``key=value`` / ``key = value`` / ``key: value`` lines; ``#`` and ``;`` start
  comments; ``[section]`` headers and ``---`` are ignored; ``[a, b]`` is a list value.
* ``store_true`` keys accept ``true/yes/1`` (flag set) and ``false/no/0`` (flag absent).
* Precedence is command line > config file > defaults: a config item is dropped when the same
  option already appears on the command line.
* Config keys that no action of the parser knows are surfaced as ``--key=value`` strings in the
  ``unknown`` list of ``parse_known_args`` so the two-parser intersection in ``get_params`` works.
* ``parse_args('-c path')`` accepts a single string and splits it (used by ``load_config_file``).
* ``serialize(items)`` writes ``key = value`` lines, the format ``write_config_file`` produces.
"""
from __future__ import annotations

import argparse
import os
import re
import sys
from collections import OrderedDict
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

__all__ = ["ArgumentParser", "ConfigFileParser", "ConfigFileParserException"]

_TRUE = {"true", "yes", "1", "on"}
_FALSE = {"false", "no", "0", "off"}


class ConfigFileParserException(Exception):
    pass


class ConfigFileParser:
    """Reader/writer for the ``key = value`` config format."""

    _line_re = re.compile(
        r"^(?P<key>[^:=;\s#]+)\s*(?:(?P<equal>[:=\s])\s*(?P<value>.+?)?)?\s*(?:\s[;#]\s*(?P<comment>.*?)\s*)?$"
    )

    def parse(self, stream) -> "OrderedDict[str, object]":
        items: "OrderedDict[str, object]" = OrderedDict()
        for i, raw in enumerate(stream):
            line = raw.strip()
            if not line or line[0] in "#;" or line.startswith("---") or (line[0] == "[" and line[-1] == "]"):
                continue
            m = self._line_re.match(line)
            if m is None:
                raise ConfigFileParserException(f"Unexpected line {i} in config file: {raw!r}")
            key = m.group("key")
            value = m.group("value")
            if value is None:
                value = "true"
            value = value.strip()
            if len(value) >= 2 and value[0] == "[" and value[-1] == "]":
                inner = value[1:-1].strip()
                items[key] = [v.strip() for v in inner.split(",")] if inner else []
            else:
                if len(value) >= 2 and value[0] == value[-1] and value[0] in "\"'":
                    value = value[1:-1]
                items[key] = value
        return items

    @staticmethod
    def serialize(items: Dict[str, object]) -> str:
        out = []
        for key, value in items.items():
            if isinstance(value, (list, tuple)):
                value = "[" + ", ".join(str(v) for v in value) + "]"
            out.append(f"{key} = {value}\n")
        return "".join(out)


class ArgumentParser(argparse.ArgumentParser):
    """``argparse.ArgumentParser`` + config files, with configargparse's observable behaviour."""

    def __init__(self, *args, **kwargs):
        kwargs.setdefault("allow_abbrev", False)
        super().__init__(*args, **kwargs)
        self._config_file_parser = ConfigFileParser()
        self._config_file_actions: List[argparse.Action] = []

    # configargparse extension: ``is_config_file=True``
    def add_argument(self, *args, **kwargs):
        is_config = kwargs.pop("is_config_file", False) or kwargs.pop("is_config_file_arg", False)
        action = super().add_argument(*args, **kwargs)
        if is_config:
            self._config_file_actions.append(action)
        return action

    # ------------------------------------------------------------------ parsing
    def _config_paths(self, args: Sequence[str]) -> List[str]:
        paths = []
        for action in self._config_file_actions:
            for opt in action.option_strings:
                for i, tok in enumerate(args):
                    if tok == opt and i + 1 < len(args):
                        paths.append(args[i + 1])
                    elif tok.startswith(opt + "="):
                        paths.append(tok[len(opt) + 1:])
        return paths

    def _find_action(self, key: str) -> Optional[argparse.Action]:
        candidates = [key] if key.startswith("-") else ["--" + key, "-" + key]
        for action in self._actions:
            for opt in action.option_strings:
                if opt in candidates:
                    return action
        return None

    @staticmethod
    def _on_command_line(action: argparse.Action, args: Sequence[str]) -> bool:
        for opt in action.option_strings:
            for tok in args:
                if tok == opt or tok.startswith(opt + "="):
                    return True
        return False

    def _item_to_args(self, action: Optional[argparse.Action], key: str, value) -> List[str]:
        if action is None:
            opt = key if key.startswith("-") else "--" + key
            if isinstance(value, list):
                value = "[" + ", ".join(value) + "]"
            return [f"{opt}={value}"]
        opt = action.option_strings[-1] if action.option_strings[-1].startswith("--") else action.option_strings[0]
        if isinstance(action, (argparse._StoreTrueAction, argparse._StoreFalseAction, argparse._StoreConstAction,
                               argparse._CountAction)):
            v = str(value).strip().lower()
            if v in _TRUE:
                return [opt]
            if v in _FALSE:
                return []
            self.error(f"Unexpected value for {key}: {value!r}. Expecting 'true' or 'false'.")
        if isinstance(value, list):
            if action.nargs in (None, 1, "?"):
                return [opt, "[" + ", ".join(value) + "]"]
            return [opt] + list(value)
        return [opt, str(value)]

    def _expand_config(self, args: List[str]) -> List[str]:
        config_args: List[str] = []
        for path in self._config_paths(args):
            if not os.path.isfile(path):
                self.error(f"File not found: {path}")
            with open(path, "r") as stream:
                items = self._config_file_parser.parse(stream)
            for key, value in items.items():
                action = self._find_action(key)
                if action is not None and action in self._config_file_actions:
                    continue
                if action is not None and self._on_command_line(action, args):
                    continue
                config_args.extend(self._item_to_args(action, key, value))
        return config_args + args

    def parse_known_args(self, args=None, namespace=None):
        if args is None:
            args = sys.argv[1:]
        elif isinstance(args, str):
            args = args.split()
        else:
            args = list(args)
        full = self._expand_config(args)
        return super().parse_known_args(full, namespace)

    def parse_args(self, args=None, namespace=None):
        ns, unknown = self.parse_known_args(args, namespace)
        if unknown:
            self.error("unrecognized arguments: %s" % " ".join(unknown))
        return ns

    # ------------------------------------------------------------------ writing
    def serialize(self, items: Dict[str, object]) -> str:
        return self._config_file_parser.serialize(items)
