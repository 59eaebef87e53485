"""Known-answer tests of the CPU oracle, restating the reference's own merge-tree specs:
packages/dds/merge-tree/src/test/client.applyMsg.spec.ts and
packages/dds/merge-tree/src/test/mergeTree.markRangeRemoved.spec.ts.

Client long ids: the reference uses strings ("localUser", "remoteClient", "A", ...); here they
are doc-local indices, named by the constants below.
"""
import pytest

from fluidframework_amd import oplog as ol
from oracle_client import Msg
from replicas import make_replica, parse_dump

LOCAL, REMOTE, REMOTE2 = 0, 1, 2

KINDS = ["oracle", "host", pytest.param("gpu", marks=pytest.mark.gpu)]


@pytest.fixture(params=KINDS)
def kind(request):
    return request.param


def seg_at(client, pos: int):
    """getContainingSegment(pos) in the local perspective (visible segments only)."""
    _, segs = parse_dump(client.dump())
    p = 0
    for s in segs:
        if s["removedSeq"] is not None:
            continue
        if p <= pos < p + s["len"]:
            return s
        p += s["len"]
    return None


@pytest.fixture
def client(kind):
    # client.applyMsg.spec.ts:17-21
    c = make_replica(kind)
    c.insert_text_local(0, "hello world")
    c.start_collab(LOCAL)
    return c


def test_interleaved_inserts_annotates_deletes(client):
    # client.applyMsg.spec.ts:23-86
    changes = {}
    for i in range(100):
        ln = client.get_length()
        pos1 = ln // 2
        m6 = i % 6
        if m6 in (0, 5):
            pos2 = max((ln - pos1) // 4 - m6 + pos1, pos1 + 1)
            op = client.remove_range_local(pos1, pos2)
        elif m6 in (1, 4):
            op = client.insert_text_local(pos1, f"{i}" * (m6 + 5))
        else:
            pos2 = max((ln - pos1) // 3 - m6 + pos1, pos1 + 1)
            op = client.annotate_range_local(pos1, pos2, {"foo": f"{i}"})
        assert op is not None
        changes[i] = client.make_op_message(op, i + 1)
    for i in range(100):
        # the segments of op i's SegmentGroup: op i is local op i + 1 (getLocalSequenceNumber), so they are
        # the rows with that localSeq (insert) / localRemovedSeq (remove). The ack neither splits nor (MSN
        # 0) scours, so the rows keep their order across it.
        _, pre = parse_dump(client.dump())
        assert client.apply_msg(changes[i]) == 0
        _, post = parse_dump(client.dump())
        assert len(pre) == len(post)
        m6 = i % 6
        for a, b in zip(pre, post):
            if m6 in (0, 5) and a["flags"] & ol.DF_LRSEQ and a["localRemovedSeq"] == i + 1:
                assert b["removedSeq"] == i + 1, "removed segment has unexpected id"  # applyMsg.spec.ts:74-76
            if m6 in (1, 4) and a["flags"] & ol.DF_LSEQ and a["localSeq"] == i + 1:
                assert b["seq"] == i + 1, "inserted segment has unexpected id"  # applyMsg.spec.ts:78-81
    _, segs = parse_dump(client.dump())
    for s in segs:
        assert s["seq"] != -1 and s["ngroups"] == 0


def test_insert_text_local_ack(client):
    # client.applyMsg.spec.ts:88-98
    op = client.insert_text_local(0, "abc")
    assert seg_at(client, 0)["seq"] == -1
    client.apply_msg(client.make_op_message(op, 17))
    assert seg_at(client, 0)["seq"] == 17


def test_remove_range_local_ack(client):
    # client.applyMsg.spec.ts:100-110
    op = client.remove_range_local(0, 1)
    _, segs = parse_dump(client.dump())
    assert segs[0]["removedSeq"] == -1 and segs[0]["len"] == 1
    client.apply_msg(client.make_op_message(op, 17))
    _, segs = parse_dump(client.dump())
    assert segs[0]["removedSeq"] == 17


def test_annotate_local_ack(client):
    # client.applyMsg.spec.ts:112-127
    op = client.annotate_range_local(0, 1, {"foo": "bar"})
    assert parse_dump(client.dump())[1][0]["ngroups"] == 1
    client.apply_msg(client.make_op_message(op, 17))
    assert parse_dump(client.dump())[1][0]["ngroups"] == 0


def test_annotate_then_remove_local(client):
    # client.applyMsg.spec.ts:129-168
    end = len(client.get_text())
    a = client.annotate_range_local(0, end, {"foo": "bar"})
    r = client.remove_range_local(0, end)
    _, segs = parse_dump(client.dump())
    assert segs[0]["removedSeq"] == -1
    assert segs[0]["ngroups"] == 2
    client.apply_msg(client.make_op_message(a, 17))
    _, segs = parse_dump(client.dump())
    assert segs[0]["removedSeq"] == -1
    assert segs[0]["ngroups"] == 1
    client.apply_msg(client.make_op_message(r, 18))
    _, segs = parse_dump(client.dump())
    assert segs[0]["removedSeq"] == 18
    assert segs[0]["ngroups"] == 0


def test_multiple_interleaved_annotates(client):
    # client.applyMsg.spec.ts:170-196
    end = len(client.get_text())
    msgs = []
    seq = 0
    while end > 0:
        op = client.annotate_range_local(0, end, {"end": end, "foo": "bar"})
        seq += 1
        msgs.append(client.make_op_message(op, seq))
        end //= 2
    assert parse_dump(client.dump())[1][0]["ngroups"] == len(msgs)
    for m in msgs:
        client.apply_msg(m)
    assert parse_dump(client.dump())[1][0]["ngroups"] == 0
    assert client.error == 0


def test_overlapping_deletes(client):
    # client.applyMsg.spec.ts:198-228
    text0 = client.get_text()
    op = client.remove_range_local(0, 5)
    _, segs = parse_dump(client.dump())
    assert segs[0]["removedSeq"] == -1 and segs[0]["ngroups"] == 1
    remote = client.make_op_message(op, 17, long_client=REMOTE)
    client.apply_msg(remote)
    _, segs = parse_dump(client.dump())
    assert segs[0]["removedSeq"] == 17 and segs[0]["ngroups"] == 1
    client.apply_msg(client.make_op_message(op, 18))
    _, segs = parse_dump(client.dump())
    assert segs[0]["removedSeq"] == 17 and segs[0]["ngroups"] == 0
    assert client.get_length() == len(text0) - 5
    assert client.get_text() == text0[5:]


def run_convergence(clients, messages):
    """TestClientLogger.log/validate (testClientLogger.ts:31-87): every client applies every
    message; all texts must agree with client 0."""
    for m in messages:
        for c in clients:
            assert c.apply_msg(m) == 0
    texts = [c.get_text() for c in clients]
    assert all(t == texts[0] for t in texts), texts
    return texts[0]


def test_overlapping_insert_and_delete(client, kind):
    # client.applyMsg.spec.ts:230-259
    remote = make_replica(kind, client.interner)
    remote.insert_text_local(0, client.get_text())
    remote.start_collab(REMOTE)
    seq = 1
    init = client.make_op_message(client.insert_text_local(0, "-"), seq)
    run_convergence([client, remote], [init])
    msgs = [
        client.make_op_message(client.insert_text_local(0, "L"), 2),
        client.make_op_message(client.remove_range_local(1, 2), 3),
        remote.make_op_message(remote.insert_text_local(0, "R"), 4),
        remote.make_op_message(remote.remove_range_local(1, 2), 5),
    ]
    run_convergence([client, remote], msgs)


def three(kind, seed_text=None):
    it = ol.Interner()
    cs = []
    for k in range(3):
        c = make_replica(kind, it)
        if seed_text:
            c.insert_text_local(0, seed_text)
        c.start_collab(k)
        cs.append(c)
    return cs


def test_intersecting_insert_after_local_delete(kind):
    # client.applyMsg.spec.ts:261-290
    A, B, C = three(kind)
    msgs = [
        C.make_op_message(C.insert_text_local(0, "c"), 1),
        C.make_op_message(C.remove_range_local(0, 1), 2),
        B.make_op_message(B.insert_text_local(0, "b"), 3),
        C.make_op_message(C.insert_text_local(0, "c"), 4),
    ]
    run_convergence([A, B, C], msgs)


def test_conflicting_insert_after_shared_delete(kind):
    # client.applyMsg.spec.ts:292-320
    A, B, C = three(kind, "a")
    msgs = [
        B.make_op_message(B.insert_text_local(0, "b"), 1),
        C.make_op_message(C.remove_range_local(0, C.get_length()), 2),
        C.make_op_message(C.insert_text_local(0, "c"), 3),
    ]
    run_convergence([A, B, C], msgs)


def test_local_remove_followed_by_conflicting_insert(kind):
    # client.applyMsg.spec.ts:322-349
    A, B, C = three(kind)
    msgs = [
        C.make_op_message(C.insert_text_local(0, "c"), 1),
        B.make_op_message(B.insert_text_local(0, "b"), 2),
        C.make_op_message(C.remove_range_local(0, 1), 3),
        C.make_op_message(C.insert_text_local(0, "c"), 4),
    ]
    run_convergence([A, B, C], msgs)


def test_intersecting_insert_with_unack_insert_and_delete(kind):
    # client.applyMsg.spec.ts:351-380
    A, B, C = three(kind)
    msgs = [
        C.make_op_message(C.insert_text_local(0, "c"), 1),
        B.make_op_message(B.insert_text_local(0, "bb"), 2),
        B.make_op_message(B.remove_range_local(0, 1), 3),
    ]
    run_convergence([A, B, C], msgs)


@pytest.fixture
def hello(kind):
    # mergeTree.markRangeRemoved.spec.ts:13-27
    c = make_replica(kind)
    c.start_collab(LOCAL)
    for ch in "hello world":
        op = c.insert_text_local(c.get_length(), ch)
        c.apply_msg(c.make_op_message(op, c.current_seq + 1))
    assert c.get_text() == "hello world"
    return c


def test_mrr_local_remove_then_local_insert(hello):
    hello.remove_range_local(0, hello.get_length())
    assert hello.get_text() == ""
    hello.insert_text_local(0, "text")
    assert hello.get_text() == "text"


def test_mrr_local_insert_then_local_remove(hello):
    hello.insert_text_local(0, "text")
    assert hello.get_text() == "texthello world"
    hello.remove_range_local(0, hello.get_length())
    assert hello.get_text() == ""


def test_mrr_remote_remove_then_local_insert(hello):
    cs = hello.current_seq
    hello.apply_msg(Msg(ol.OP_REMOVE, 0, hello.get_length()).sequenced(cs + 1, cs, REMOTE))
    assert hello.get_text() == ""
    hello.insert_text_local(0, "text")
    assert hello.get_text() == "text"


def test_mrr_local_remove_then_remote_insert(hello):
    hello.remove_range_local(0, hello.get_length())
    assert hello.get_text() == ""
    cs = hello.current_seq
    hello.apply_msg(Msg(ol.OP_INSERT, 0, text="text").sequenced(cs + 1, cs, REMOTE))
    assert hello.get_text() == "text"


def test_mrr_remote_remove_then_remote_insert(hello):
    cs = hello.current_seq
    rm = Msg(ol.OP_REMOVE, 0, hello.get_length()).sequenced(cs + 1, cs, REMOTE2)
    ins = Msg(ol.OP_INSERT, 0, text="text").sequenced(cs + 2, cs, REMOTE)
    hello.apply_msg(rm)
    hello.apply_msg(ins)
    assert hello.get_text() == "text"


def test_mrr_remote_insert_then_remote_remove(hello):
    cs = hello.current_seq
    ins = Msg(ol.OP_INSERT, 0, text="text").sequenced(cs + 1, cs, REMOTE)
    rm = Msg(ol.OP_REMOVE, 0, hello.get_length()).sequenced(cs + 2, cs, REMOTE2)
    hello.apply_msg(ins)
    hello.apply_msg(rm)
    assert hello.get_text() == "text"
