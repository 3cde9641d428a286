"""TensorBoard event writer: TFRecord framing (masked CRC32C) and Event/Summary protobuf encoding,
checked against an independent protobuf decoder built from the tensorflow ``event.proto`` field
numbers (tensorboard itself is not installed here)."""
import glob
import struct

import pytest

from ml_recipe_distributed_pytorch_amd.utils import tb


def test_crc32c_known_vectors(host_lib):
    assert tb.crc32c(b"123456789") == 0xE3069283
    assert tb._crc32c_py(b"123456789") == 0xE3069283
    data = bytes(range(256)) * 17
    assert tb.crc32c(data) == tb._crc32c_py(data)


def _event_class():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    fdp = descriptor_pb2.FileDescriptorProto(name="hq_event_test.proto", package="hqtest", syntax="proto3")
    val = fdp.message_type.add(name="Value")
    val.field.add(name="tag", number=1, type=9, label=1)
    val.field.add(name="simple_value", number=2, type=2, label=1)
    summ = fdp.message_type.add(name="Summary")
    summ.field.add(name="value", number=1, type=11, label=3, type_name=".hqtest.Value")
    ev = fdp.message_type.add(name="Event")
    ev.field.add(name="wall_time", number=1, type=1, label=1)
    ev.field.add(name="step", number=2, type=3, label=1)
    ev.field.add(name="file_version", number=3, type=9, label=1)
    ev.field.add(name="summary", number=5, type=11, label=1, type_name=".hqtest.Summary")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("hqtest.Event"))


def test_writer_roundtrip(tmp_path):
    w = tb.SummaryWriter(str(tmp_path))
    for step in range(5):
        w.add_scalar("train/loss", 1.0 / (step + 1), global_step=step)
        w.add_scalar("perf/samples_per_sec", 100.0 * step, global_step=step)
    w.close()
    files = glob.glob(str(tmp_path / "events.out.tfevents.*"))
    assert len(files) == 1
    ev = tb.read_events(files[0])
    losses = [(s, v) for s, t, v in ev if t == "train/loss"]
    assert [s for s, _ in losses] == list(range(5))
    assert losses[2][1] == pytest.approx(1 / 3, rel=1e-6)

    Event = _event_class()
    data = open(files[0], "rb").read()
    pos, parsed = 0, []
    while pos < len(data):
        (n,) = struct.unpack_from("<Q", data, pos)
        e = Event()
        e.ParseFromString(data[pos + 12:pos + 12 + n])
        parsed.append(e)
        pos += 16 + n
    assert parsed[0].file_version.startswith("brain.Event:")
    vals = [(e.step, v.tag, v.simple_value) for e in parsed[1:] for v in e.summary.value]
    assert ("train/loss", 4) in {(t, s) for s, t, _ in vals}
    assert len(vals) == 10
