"""
Settings DSL (L4): a pydantic model that renders to ``argparse`` and loads
from JSON.  API-compatible with the reference ``config/base.py``
(reference: config/base.py:15-87): ``S``/``Setting``, ``C``/``Choice``,
``_``/``Item``, ``Validator``, ``to_argparse``, ``from_argparse``,
``from_argv``, ``dict()``, ``json(indent=...)``, ``parse_file``.

Written against the pydantic **v2** API (the reference used v1-only
``pydantic.validators.bool_validator`` / ``__fields__`` internals and fails to
import under pydantic 2).  Nested setting groups work (the
reference's name-mangled ``__top`` keyword crashed them).
"""
import argparse
import json
from typing import Literal, get_args, get_origin

from pydantic import BaseModel, ConfigDict, Field

try:  # pydantic v2
    from pydantic import field_validator as _field_validator
except ImportError:  # pragma: no cover
    _field_validator = None

_TRUE = {"1", "on", "t", "true", "y", "yes"}
_FALSE = {"0", "off", "f", "false", "n", "no"}


def bool_validator(value):
    """Parse booleans the way pydantic v1's ``bool_validator`` did."""
    if isinstance(value, bool):
        return value
    if isinstance(value, (int, float)) and value in (0, 1):
        return bool(value)
    text = str(value).strip().lower()
    if text in _TRUE:
        return True
    if text in _FALSE:
        return False
    raise argparse.ArgumentTypeError(f"value could not be parsed to a boolean: {value!r}")


def _is_model(tp):
    return isinstance(tp, type) and issubclass(tp, BaseModel)


def _choice_converter(name, choices):
    by_text = {str(c): c for c in choices}

    def convert(arg):
        if arg in by_text:
            return by_text[arg]
        raise ValueError(arg)

    convert.__name__ = name
    return convert


class ArgparseCompatibleBaseModel(BaseModel):
    """pydantic model <-> argparse bridge.  Unknown keys are rejected."""

    model_config = ConfigDict(extra="forbid", validate_assignment=True,
                              protected_namespaces=())

    # ---- argparse -----------------------------------------------------------
    @classmethod
    def from_argparse(cls, namespace, _top=True):
        if not isinstance(namespace, dict):
            namespace = vars(namespace)
        kwargs = {}
        for name, field in cls.model_fields.items():
            if _is_model(field.annotation):
                kwargs[name] = ArgparseCompatibleBaseModel.from_argparse.__func__(
                    field.annotation, namespace, _top=False)
            elif name in namespace:
                kwargs[name] = namespace.pop(name)
        assert not (_top and namespace), str(namespace)
        return cls(**kwargs)

    @classmethod
    def _argparse_kwargs(cls, name, field, suppress_defaults=False):
        tp = field.annotation
        default = None if field.is_required() else field.default
        help_text = field.description or ""
        kw = dict(dest=name, type=tp, default=default, help=help_text,
                  required=field.is_required() and not suppress_defaults)
        if get_origin(tp) is Literal:
            choices = tuple(get_args(tp))
            kw.update(type=_choice_converter(name, choices), choices=choices,
                      metavar="{" + ", ".join(map(str, choices)) + "}")
        elif tp is bool:
            kw.update(type=bool_validator, metavar="{true, false}")
        if suppress_defaults:
            # Only flags given on the command line reach the namespace; the
            # default is still shown in --help.
            kw["help"] = f"{help_text} (default: {default})"
            kw["default"] = argparse.SUPPRESS
        return kw

    @classmethod
    def to_argparse(cls, parser_or_group=None, _suppress_defaults=False):
        if parser_or_group is None:
            parser_or_group = argparse.ArgumentParser(
                formatter_class=argparse.ArgumentDefaultsHelpFormatter)
        for name, field in cls.model_fields.items():
            if _is_model(field.annotation):
                group = parser_or_group.add_argument_group(name)
                ArgparseCompatibleBaseModel.to_argparse.__func__(
                    field.annotation, group, _suppress_defaults)
                continue
            parser_or_group.add_argument(
                "--" + name, **cls._argparse_kwargs(name, field, _suppress_defaults))
        return parser_or_group

    @classmethod
    def from_argv(cls, argv=None):
        return cls.from_argparse(cls.to_argparse().parse_args(argv))

    # ---- pydantic-v1 style conveniences (kept for API compatibility) -------
    def dict(self, **kwargs):  # noqa: A003 - v1 API name
        return self.model_dump(**kwargs)

    def json(self, indent=None, **kwargs):
        return json.dumps(self.model_dump(**kwargs), indent=indent)

    @classmethod
    def parse_obj(cls, obj):
        return cls.model_validate(obj)

    @classmethod
    def parse_file(cls, path):
        with open(path, "r") as f:
            return cls.model_validate(json.load(f))

    @classmethod
    def field_names(cls):
        return list(cls.model_fields)


S = Setting = ArgparseCompatibleBaseModel


def choice(*args):
    """``x: C('a', 'b') = _('a', '...')`` -> a ``Literal`` typed field."""
    return Literal.__getitem__(args)


C = Choice = choice


def item(default, description=None):
    return Field(default, description=description)


_ = Item = item


def validator(*fields, **kwargs):
    """v1-style ``@validator('field')`` mapped onto pydantic v2."""
    kwargs.pop("allow_reuse", None)
    pre = kwargs.pop("pre", False)
    return _field_validator(*fields, mode="before" if pre else "after", **kwargs)


Validator = validator

__all__ = (
    'ArgparseCompatibleBaseModel', 'Setting', 'S',
    'choice', 'Choice', 'C',
    'item', 'Item', '_',
    'validator', 'Validator', 'bool_validator',
)
