"""Build protobuf message classes from a compact in-code schema (no protoc in the image).

A schema is a dict of message specs; each field is ``(name, number, type[, label])`` where
``type`` is a scalar name (``string``, ``int64``, ``float`` ...), ``.pkg.Message`` /
``.pkg.Enum`` for references, and label is ``opt`` (proto3 singular, default), ``rep``
or ``map:<key>:<value>``. Field numbers and names are the wire contract, so building
the descriptor in code is byte-compatible with protoc output for the same .proto.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_T = descriptor_pb2.FieldDescriptorProto
SCALARS = {
    "double": _T.TYPE_DOUBLE, "float": _T.TYPE_FLOAT, "int64": _T.TYPE_INT64,
    "uint64": _T.TYPE_UINT64, "int32": _T.TYPE_INT32, "fixed64": _T.TYPE_FIXED64,
    "fixed32": _T.TYPE_FIXED32, "bool": _T.TYPE_BOOL, "string": _T.TYPE_STRING,
    "bytes": _T.TYPE_BYTES, "uint32": _T.TYPE_UINT32, "sint32": _T.TYPE_SINT32,
    "sint64": _T.TYPE_SINT64,
}

_POOL = descriptor_pool.DescriptorPool()
_BUILT: Dict[str, Dict[str, type]] = {}


def _ensure_timestamp() -> None:
    name = "google/protobuf/timestamp.proto"
    try:
        _POOL.FindFileByName(name)
        return
    except KeyError:
        pass
    fd = descriptor_pb2.FileDescriptorProto(name=name, package="google.protobuf", syntax="proto3")
    m = fd.message_type.add(name="Timestamp")
    m.field.add(name="seconds", number=1, type=_T.TYPE_INT64, label=_T.LABEL_OPTIONAL)
    m.field.add(name="nanos", number=2, type=_T.TYPE_INT32, label=_T.LABEL_OPTIONAL)
    _POOL.Add(fd)


def _add_field(msg, fd_proto, name: str, number: int, ftype: str, label: str, pkg: str) -> None:
    f = msg.field.add(name=name, number=number, json_name=_json_name(name))
    if label.startswith("map:"):
        _, kt, vt = label.split(":")
        entry_name = "".join(p.capitalize() for p in name.split("_")) + "Entry"
        e = msg.nested_type.add(name=entry_name)
        e.options.map_entry = True
        for n, num, t in (("key", 1, kt), ("value", 2, vt)):
            ef = e.field.add(name=n, number=num, label=_T.LABEL_OPTIONAL, json_name=n)
            _set_type(ef, t)
        f.label = _T.LABEL_REPEATED
        f.type = _T.TYPE_MESSAGE
        f.type_name = f".{pkg}.{msg.name}.{entry_name}"
        return
    f.label = _T.LABEL_REPEATED if label == "rep" else _T.LABEL_OPTIONAL
    _set_type(f, ftype)


def _set_type(f, ftype: str) -> None:
    if ftype in SCALARS:
        f.type = SCALARS[ftype]
    elif ftype.startswith("enum:"):
        f.type = _T.TYPE_ENUM
        f.type_name = ftype[5:]
    else:
        f.type = _T.TYPE_MESSAGE
        f.type_name = ftype


def _json_name(name: str) -> str:
    parts = name.split("_")
    return parts[0] + "".join(p.capitalize() for p in parts[1:])


def build_file(file_name: str, package: str, messages: Dict[str, Sequence[Tuple]],
               enums: Dict[str, Sequence[Tuple[str, int]]] = None,
               services: Dict[str, Sequence[Tuple[str, str, str]]] = None,
               deps: List[str] = None, syntax: str = "proto3") -> Dict[str, type]:
    """Register a file in the private pool; return {message name: class}."""
    if file_name in _BUILT:
        return _BUILT[file_name]
    deps = deps or []
    if "google/protobuf/timestamp.proto" in deps:
        _ensure_timestamp()
    fd = descriptor_pb2.FileDescriptorProto(name=file_name, package=package, syntax=syntax)
    fd.dependency.extend(deps)
    for ename, values in (enums or {}).items():
        e = fd.enum_type.add(name=ename)
        for vname, vnum in values:
            e.value.add(name=vname, number=vnum)
    for mname, flds in messages.items():
        m = fd.message_type.add(name=mname)
        for spec in flds:
            name, number, ftype = spec[0], spec[1], spec[2]
            label = spec[3] if len(spec) > 3 else "opt"
            _add_field(m, fd, name, number, ftype, label, package)
    for sname, methods in (services or {}).items():
        s = fd.service.add(name=sname)
        for spec in methods:
            mname, itype, otype = spec[:3]
            mode = spec[3] if len(spec) > 3 else ""
            s.method.add(name=mname, input_type=f".{package}.{itype}", output_type=f".{package}.{otype}",
                         client_streaming=mode in ("client_stream", "bidi"),
                         server_streaming=mode in ("server_stream", "bidi"))
    _POOL.Add(fd)
    out = {}
    for mname in messages:
        desc = _POOL.FindMessageTypeByName(f"{package}.{mname}")
        out[mname] = message_factory.GetMessageClass(desc)
    _BUILT[file_name] = out
    return out


def enum_values(full_name: str) -> Dict[str, int]:
    d = _POOL.FindEnumTypeByName(full_name)
    return {v.name: v.number for v in d.values}


def file_descriptor(file_name: str):
    return _POOL.FindFileByName(file_name)


def file_descriptor_proto_bytes(file_name: str) -> bytes:
    p = descriptor_pb2.FileDescriptorProto()
    _POOL.FindFileByName(file_name).CopyToProto(p)
    return p.SerializeToString()


def file_containing_symbol(symbol: str) -> str:
    return _POOL.FindFileContainingSymbol(symbol).name


def timestamp_class():
    _ensure_timestamp()
    return message_factory.GetMessageClass(_POOL.FindMessageTypeByName("google.protobuf.Timestamp"))
