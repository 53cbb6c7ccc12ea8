"""The subset of ``onnx.proto`` (IR v8/9) this framework reads and writes, built in code.

``onnx`` / ``onnxruntime`` are not installable here, so models are written through these
classes and read by the C++ reader in ``csrc/runtime/onnx_reader.cpp``. Nested ONNX types
(``TypeProto.Tensor``, ``TensorShapeProto.Dimension``) are declared top-level with
``_`` names: nesting is invisible on the wire, field numbers are ONNX's.
"""
from __future__ import annotations

from ..proto.builder import build_file

PKG = "onnx"
MESSAGES = {
    "StringStringEntryProto": [("key", 1, "string"), ("value", 2, "string")],
    "OperatorSetIdProto": [("domain", 1, "string"), ("version", 2, "int64")],
    "TensorProto": [
        ("dims", 1, "int64", "rep"), ("data_type", 2, "int32"),
        ("float_data", 4, "float", "rep"), ("int32_data", 5, "int32", "rep"),
        ("string_data", 6, "bytes", "rep"), ("int64_data", 7, "int64", "rep"),
        ("name", 8, "string"), ("doc_string", 12, "string"), ("raw_data", 9, "bytes"),
        ("double_data", 10, "double", "rep"), ("uint64_data", 11, "uint64", "rep"),
    ],
    "TensorShapeProto_Dimension": [("dim_value", 1, "int64"), ("dim_param", 2, "string")],
    "TensorShapeProto": [("dim", 1, ".onnx.TensorShapeProto_Dimension", "rep")],
    "TypeProto_Tensor": [("elem_type", 1, "int32"), ("shape", 2, ".onnx.TensorShapeProto")],
    "TypeProto": [("tensor_type", 1, ".onnx.TypeProto_Tensor"), ("denotation", 6, "string")],
    "ValueInfoProto": [("name", 1, "string"), ("type", 2, ".onnx.TypeProto"),
                       ("doc_string", 3, "string")],
    "AttributeProto": [
        ("name", 1, "string"), ("f", 2, "float"), ("i", 3, "int64"), ("s", 4, "bytes"),
        ("t", 5, ".onnx.TensorProto"), ("floats", 7, "float", "rep"),
        ("ints", 8, "int64", "rep"), ("strings", 9, "bytes", "rep"),
        ("tensors", 10, ".onnx.TensorProto", "rep"), ("doc_string", 13, "string"),
        ("type", 20, "int32"),
    ],
    "NodeProto": [
        ("input", 1, "string", "rep"), ("output", 2, "string", "rep"), ("name", 3, "string"),
        ("op_type", 4, "string"), ("attribute", 5, ".onnx.AttributeProto", "rep"),
        ("doc_string", 6, "string"), ("domain", 7, "string"),
    ],
    "GraphProto": [
        ("node", 1, ".onnx.NodeProto", "rep"), ("name", 2, "string"),
        ("initializer", 5, ".onnx.TensorProto", "rep"), ("doc_string", 10, "string"),
        ("input", 11, ".onnx.ValueInfoProto", "rep"), ("output", 12, ".onnx.ValueInfoProto", "rep"),
        ("value_info", 13, ".onnx.ValueInfoProto", "rep"),
    ],
    "ModelProto": [
        ("ir_version", 1, "int64"), ("producer_name", 2, "string"),
        ("producer_version", 3, "string"), ("domain", 4, "string"), ("model_version", 5, "int64"),
        ("doc_string", 6, "string"), ("graph", 7, ".onnx.GraphProto"),
        ("opset_import", 8, ".onnx.OperatorSetIdProto", "rep"),
        ("metadata_props", 14, ".onnx.StringStringEntryProto", "rep"),
    ],
}

M = build_file("onnx/onnx-subset.proto", PKG, MESSAGES, syntax="proto2")

# TensorProto.DataType
FLOAT, UINT8, INT8, INT32, INT64, STRING, BOOL, FLOAT16, DOUBLE, BFLOAT16 = 1, 2, 3, 6, 7, 8, 9, 10, 11, 16
# AttributeProto.AttributeType
A_FLOAT, A_INT, A_STRING, A_TENSOR, A_FLOATS, A_INTS, A_STRINGS = 1, 2, 3, 4, 6, 7, 8

ModelProto = M["ModelProto"]
GraphProto = M["GraphProto"]
NodeProto = M["NodeProto"]
TensorProto = M["TensorProto"]
AttributeProto = M["AttributeProto"]
ValueInfoProto = M["ValueInfoProto"]
