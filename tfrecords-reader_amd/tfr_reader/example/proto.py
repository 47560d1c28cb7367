"""tf.train.Example message classes for the optional "protobuf" decoder, built at run time.

The schema is the public tensorflow/core/example/{example,feature}.proto (proto3, packed repeated
numerics). It is declared here programmatically so no generated code is needed.
"""

from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_F = descriptor_pb2.FieldDescriptorProto


def _file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name="tfrg_tf_example.proto", package="tfrg.tf", syntax="proto3")

    def msg(name, fields, nested=(), oneofs=()):
        m = fd.message_type.add(name=name)
        for o in oneofs:
            m.oneof_decl.add(name=o)
        for fname, num, typ, label, type_name, oneof in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if type_name:
                f.type_name = type_name
            if oneof is not None:
                f.oneof_index = oneof
        for n in nested:
            m.nested_type.add().CopyFrom(n)
        return m

    rep, opt = _F.LABEL_REPEATED, _F.LABEL_OPTIONAL
    msg("BytesList", [("value", 1, _F.TYPE_BYTES, rep, None, None)])
    msg("FloatList", [("value", 1, _F.TYPE_FLOAT, rep, None, None)])
    msg("Int64List", [("value", 1, _F.TYPE_INT64, rep, None, None)])
    msg(
        "Feature",
        [
            ("bytes_list", 1, _F.TYPE_MESSAGE, opt, ".tfrg.tf.BytesList", 0),
            ("float_list", 2, _F.TYPE_MESSAGE, opt, ".tfrg.tf.FloatList", 0),
            ("int64_list", 3, _F.TYPE_MESSAGE, opt, ".tfrg.tf.Int64List", 0),
        ],
        oneofs=("kind",),
    )
    entry = descriptor_pb2.DescriptorProto(name="FeatureEntry")
    entry.field.add(name="key", number=1, type=_F.TYPE_STRING, label=opt)
    entry.field.add(name="value", number=2, type=_F.TYPE_MESSAGE, label=opt, type_name=".tfrg.tf.Feature")
    entry.options.map_entry = True
    msg("Features", [("feature", 1, _F.TYPE_MESSAGE, rep, ".tfrg.tf.Features.FeatureEntry", None)], nested=[entry])
    msg("Example", [("features", 1, _F.TYPE_MESSAGE, opt, ".tfrg.tf.Features", None)])
    return fd


_pool = descriptor_pool.DescriptorPool()
_pool.Add(_file())


def _cls(name: str):
    return message_factory.GetMessageClass(_pool.FindMessageTypeByName(f"tfrg.tf.{name}"))


Example = _cls("Example")
Features = _cls("Features")
Feature = _cls("Feature")
BytesList = _cls("BytesList")
FloatList = _cls("FloatList")
Int64List = _cls("Int64List")
