"""Plain value classes without ``dataclasses``.

``import dataclasses`` pulls in ``inspect`` (tokenize, linecache, ast ...): ~3-4 ms on the MI355X
host and ~10 ms on slower CPUs, paid by every ``./setup.sh`` before the bring-up starts. The
value types on that path (provider.base, config, provision, playbook, models.hostinfo) need
only the basics, which this module provides with no imports at all:

* ``@record`` / ``@record(frozen=True)``: ``__init__`` from the class annotations in order
  (defaults from class attributes, ``field(default_factory=...)``), ``__repr__``, ``__eq__``,
  and for frozen records immutability and ``__hash__`` (eq-only records are unhashable, as with
  dataclasses);
* ``fields(cls_or_obj)`` (objects with ``.name``), ``asdict(obj)`` (deep, like
  ``dataclasses.asdict``).
"""
from __future__ import annotations

_MISSING = object()


class Field:
    __slots__ = ("name", "default", "default_factory")

    def __init__(self, default=_MISSING, default_factory=_MISSING):
        self.name = ""
        self.default = default
        self.default_factory = default_factory

    def __repr__(self) -> str:
        return f"Field({self.name!r})"


def field(*, default=_MISSING, default_factory=_MISSING) -> Field:
    return Field(default, default_factory)


def _collect(cls) -> tuple[Field, ...]:
    out: dict[str, Field] = {}
    for base in reversed(cls.__mro__[1:]):
        for f in getattr(base, "__record_fields__", ()):
            out[f.name] = f
    for name in cls.__dict__.get("__annotations__", {}):
        if name.startswith("__"):
            continue
        v = cls.__dict__.get(name, _MISSING)
        f = v if isinstance(v, Field) else Field(default=v)
        f.name = name
        if isinstance(v, Field):
            if v.default is _MISSING:
                try:
                    delattr(cls, name)
                except AttributeError:
                    pass
            else:
                setattr(cls, name, v.default)
        out[name] = f
    return tuple(out.values())


def record(cls=None, *, frozen: bool = False):
    def wrap(cls):
        flds = _collect(cls)
        names = tuple(f.name for f in flds)
        cls.__record_fields__ = flds
        setter = object.__setattr__

        def __init__(self, *args, **kw):
            if len(args) > len(flds):
                raise TypeError(f"{cls.__name__}() takes {len(flds)} positional arguments but {len(args)} were given")
            for i, f in enumerate(flds):
                if i < len(args):
                    if f.name in kw:
                        raise TypeError(f"{cls.__name__}() got multiple values for argument {f.name!r}")
                    v = args[i]
                elif f.name in kw:
                    v = kw.pop(f.name)
                elif f.default_factory is not _MISSING:
                    v = f.default_factory()
                elif f.default is not _MISSING:
                    v = f.default
                else:
                    raise TypeError(f"{cls.__name__}() missing required argument: {f.name!r}")
                setter(self, f.name, v)
            if kw:
                raise TypeError(f"{cls.__name__}() got an unexpected keyword argument {next(iter(kw))!r}")
            post = getattr(self, "__post_init__", None)
            if post is not None:
                post()

        def __repr__(self):
            return f"{cls.__qualname__}(" + ", ".join(f"{n}={getattr(self, n)!r}" for n in names) + ")"

        def __eq__(self, other):
            if other.__class__ is not self.__class__:
                return NotImplemented
            return all(getattr(self, n) == getattr(other, n) for n in names)

        cls.__init__ = __init__
        if "__repr__" not in cls.__dict__:
            cls.__repr__ = __repr__
        if "__eq__" not in cls.__dict__:
            cls.__eq__ = __eq__
        if frozen:
            def __setattr__(self, name, value):
                raise AttributeError(f"cannot assign to field {name!r} of frozen {cls.__name__}")

            def __hash__(self):
                return hash(tuple(getattr(self, n) for n in names))

            cls.__setattr__ = __setattr__
            cls.__delattr__ = __setattr__
            cls.__hash__ = __hash__
        elif "__hash__" not in cls.__dict__:
            cls.__hash__ = None
        return cls

    return wrap if cls is None else wrap(cls)


def fields(obj) -> tuple[Field, ...]:
    return obj.__record_fields__


def is_record(obj) -> bool:
    return hasattr(type(obj), "__record_fields__") and not isinstance(obj, type)


def asdict(obj):
    """Deep conversion to plain dicts / lists (records nested in lists, tuples and dicts too)."""
    if is_record(obj):
        return {f.name: asdict(getattr(obj, f.name)) for f in obj.__record_fields__}
    if isinstance(obj, list):
        return [asdict(v) for v in obj]
    if isinstance(obj, tuple):
        return type(obj)(asdict(v) for v in obj) if not hasattr(obj, "_fields") else type(obj)(*(asdict(v) for v in obj))
    if isinstance(obj, dict):
        return {asdict(k): asdict(v) for k, v in obj.items()}
    if isinstance(obj, (set, frozenset)):
        return type(obj)(asdict(v) for v in obj)
    return obj
