"""CPU tests of the wire formats (mcs_amd/wire.py).

The reference has no tests or fixtures for its wire records and Go is absent here, so the expected
bytes below are derived by hand from the rules the module restates (Go 1.21 encoding/json, the
proto3 binary encoding of protobuf-go v1.34.1) and from the reference structs
(scheduler.go:65-73, cluster.go:14-24,127-138, trader.proto:20-49, resource-channel.proto:27-52);
each derivation is written beside its vector.  The /newClient snapshot is cross-checked against the
FIFO oracle's placements for the same input."""
import struct

import numpy as np
import pytest

import oracle_ref as O
from mcs_amd import Cluster, GenParams, gen_streams_host, replicate, uniform_cluster
from mcs_amd import wire as W
from mcs_amd.cluster import Node


# ---- Job JSON ---------------------------------------------------------------------------------
CLIENT_JOB = (b'{"Id":7,"MemoryNeeded":12000,"CoresNeeded":16,"State":"","Duration":300000000000,'
              b'"WaitTime":"0001-01-01T00:00:00Z","Ownership":""}\n')


def test_encode_job_is_go_encoder_output():
    # client.go:94-101 sets Id, CoresNeeded, Duration (whole seconds), MemoryNeeded; the rest stays
    # zero: "" strings and the zero time.Time; Encoder.Encode appends "\n"
    assert W.encode_job(W.Job(Id=7, MemoryNeeded=12000, CoresNeeded=16, Duration=300 * W.NS_PER_S)) == CLIENT_JOB


def test_decode_job_round_trip_and_go_rules():
    assert W.encode_job(W.decode_job(CLIENT_JOB)) == CLIENT_JOB
    j = W.decode_job(b' \n{"id":3,"coresneeded":2,"MEMORYNEEDED":5,"duration":2000000000,"extra":[1,{"a":null}]} trailing')
    assert (j.Id, j.CoresNeeded, j.MemoryNeeded, j.Duration) == (3, 2, 5, 2 * W.NS_PER_S)
    assert W.decode_job(b'{"Id":1,"id":2}').Id == 2          # keys assign in order: the last wins
    assert W.decode_job(b'{"id":2,"Id":1}').Id == 1
    assert W.decode_job(b'{"Id":null,"State":null}') == W.Job()  # null leaves the zero value
    assert W.decode_job(b"null") == W.Job()                       # Decode(&j) of null: no error
    assert W.decode_job(b'{"Duration":-5}').Duration == -5        # int64 accepts negatives
    assert W.decode_job('{"Id":18446744073709551615}').Id == (1 << 64) - 1


@pytest.mark.parametrize("body", [
    b'{"Id":-1}', b'{"Id":1.0}', b'{"Id":1e3}', b'{"Id":"1"}', b'{"Id":true}', b'{"Id":[1]}',
    b'{"Id":18446744073709551616}', b'{"State":5}', b'{"Duration":1.5}', b'{"Duration":9223372036854775808}',
    b'{"WaitTime":"yesterday"}', b'{"WaitTime":5}', b'{"WaitTime":"2024-02-30T00:00:00Z"}', b'[1]', b'"x"',
    b"", b"   ", b'{"Id":NaN}', b'{"Id":1', b'{"Id":01}',
])
def test_decode_job_rejects_like_the_handler(body):
    with pytest.raises(W.WireError):  # the "/" and "/delay" handlers answer 400 (server.go:32-35,61-64)
        W.decode_job(body)


def test_time_and_string_encoding():
    # RFC 3339 in, RFC 3339 with nanoseconds out: ".500" trims to ".5", offset +00:00 prints Z
    j = W.decode_job(b'{"WaitTime":"2024-05-01T10:00:00.500+00:00"}')
    assert j.WaitTime == "2024-05-01T10:00:00.5Z"
    assert W.decode_job(b'{"WaitTime":"2024-05-01T10:00:00.000-05:30"}').WaitTime == "2024-05-01T10:00:00-05:30"
    # HTML escaping of <, >, & and U+2028; control characters as \n or \u00XX (Go 1.21 has no \b, \f)
    out = W.encode_job(W.Job(State="<a&b>", Ownership='q"\\\n\x01\x08 é'))
    assert (b'"State":"\\u003ca\\u0026b\\u003e"' in out and
            b'"Ownership":"q\\"\\\\\\n\\u0001\\u0008\\u2028\xc3\xa9"' in out)


def test_go_float32_formatting():
    cases = [(0.0, "0"), (-0.0, "-0"), (1.0, "1"), (0.1, "0.1"), (1 / 3, "0.33333334"), (1e-7, "1e-7"),
             (1.5e-7, "1.5e-7"), (1e-6, "0.000001"), (123456789.0, "123456790"), (1e21, "1e+21"), (0.8, "0.8"),
             (16777217.0, "16777216"), (-2.5e-9, "-2.5e-9"), (3.4028235e38, "3.4028235e+38")]
    for x, want in cases:
        assert W.go_float32(x) == want, x
    with pytest.raises(W.WireError):
        W.go_float32(float("nan"))


def test_streams_from_posts_round_trip_and_engine_rules():
    arrays = replicate(uniform_cluster(5), 3)
    s = gen_streams_host(GenParams(seed=9), arrays, 300)
    posts = W.posts_from_streams(s)
    assert posts[0][0][1].startswith(b'{"Id":0,')
    back, ids = W.streams_from_posts(posts)
    for f in ("arrival", "dur", "cores", "mem", "job_off"):
        np.testing.assert_array_equal(getattr(back, f), getattr(s, f), err_msg=f)
    np.testing.assert_array_equal(ids[2], np.arange(300))
    half = W.encode_job(W.Job(Id=1, Duration=1_500_000_000))
    with pytest.raises(W.WireError, match="D8"):
        W.streams_from_posts([[(0, half)]])
    big = W.encode_job(W.Job(Id=1, CoresNeeded=1 << 32))
    with pytest.raises(W.WireError, match="D7"):
        W.streams_from_posts([[(0, big)]])
    with pytest.raises(W.WireError, match="arrival order"):
        W.streams_from_posts([[(5, CLIENT_JOB), (4, CLIENT_JOB)]])


# ---- /newClient cluster snapshot --------------------------------------------------------------
def two_node_cluster():
    nodes = [Node(Id=i, Type="physical", Memory=100, Cores=4, MemoryAvailable=100, CoresAvailable=4) for i in (1, 2)]
    return Cluster(Id=7, Nodes=nodes, URL="http://x")


# jobs (arrival, dur, cores, mem) with Go Ids 10, 9, 11, 2 (hand trace under SFIFO, A.2):
#   t=0: j0 -> node 0 [0,5); j1 -> node 1 [0,2); j2 (2 cores) fits nowhere -> WaitQueue head;
#        retried when j1 finishes: t=2 release, j2 -> node 1 [2,3), State "Waiting"; sleep 1 s
#   t=3: j2 released; j3 (0 cores, 5 mem) -> node 0 [3,12)
JOBS = np.array([[0, 5, 4, 10], [0, 2, 3, 10], [0, 1, 2, 10], [0, 9, 0, 5]], dtype=np.uint32)
IDS = [10, 9, 11, 2]


def snapshot(t, **kw):
    cl = two_node_cluster()
    a, d, c, m = JOBS.T
    node, start, fin, _ = O.fifo_run([4, 4], [100, 100], a, d, c, m)
    assert list(node) == [0, 1, 1, 0] and list(start) == [0, 0, 2, 3] and list(fin) == [5, 2, 3, 12]
    return W.cluster_snapshot(cl, t, a, d, c, m, node, start, fin, ids=IDS, **kw)


def job_js(i, state=""):
    a, d, c, m = (int(x) for x in JOBS[i])
    return ('{"Id":%d,"MemoryNeeded":%d,"CoresNeeded":%d,"State":"%s","Duration":%d,'
            '"WaitTime":"0001-01-01T00:00:00Z","Ownership":""}' % (IDS[i], m, c, state, d * W.NS_PER_S))


def node_js(nid, mem_av, cores_av, running):
    return ('{"Id":%d,"Type":"physical","URL":"","Memory":100,"Cores":4,"MemoryAvailable":%d,"CoresAvailable":%d,'
            '"RunningJobs":{%s},"Time":0}' % (nid, mem_av, cores_av, running))


def test_snapshot_at_t2_waiting_job_running():
    want = ('{"Id":7,"Nodes":[' + node_js(1, 90, 0, '"10":' + job_js(0)) + "," +
            node_js(2, 90, 2, '"11":' + job_js(2, "Waiting")) +
            '],"URL":"http://x","TotalMemory":200,"TotalCore":8,"MemoryUtilization":20,"CoreUtilization":6}\n')
    assert snapshot(2).decode() == want


def test_snapshot_at_t3_map_keys_sorted_as_strings():
    # node 0 runs Ids 10 and 2: encoding/json sorts map keys as strings, "10" < "2"
    want = ('{"Id":7,"Nodes":[' + node_js(1, 85, 0, '"10":' + job_js(0) + ',"2":' + job_js(3)) + "," +
            node_js(2, 100, 4, "") +
            '],"URL":"http://x","TotalMemory":200,"TotalCore":8,"MemoryUtilization":15,"CoreUtilization":4}\n')
    assert snapshot(3).decode() == want
    unsampled = snapshot(3, sampled=False).decode()
    assert unsampled.endswith('"MemoryUtilization":0,"CoreUtilization":0}\n')


def test_snapshot_conservation_on_a_seeded_run():
    """Free counters at any t equal the spec minus the needs of the jobs running at t; after the
    last finish every node is back to its JSON availability."""
    spec = Cluster.load(__import__("os").path.join(__import__("os").path.dirname(__import__("os").path.dirname(
        __import__("os").path.abspath(__file__))), "assets", "cluster_small.json"))
    s = gen_streams_host(GenParams(seed=3), replicate(spec, 1), 400)
    node, start, fin, _ = O.fifo_run([32] * 5, [24000] * 5, s.arrival, s.dur, s.cores, s.mem)
    import json
    for t in (0, 500, 1000, int(fin.max())):
        snap = json.loads(W.cluster_snapshot(spec, t, s.arrival, s.dur, s.cores, s.mem, node, start, fin))
        for k, nd in enumerate(snap["Nodes"]):
            run = (node == k) & (start <= t) & (fin > t)
            assert nd["CoresAvailable"] == 32 - int(s.cores[run].sum())
            assert nd["MemoryAvailable"] == 24000 - int(s.mem[run].sum())
            assert sorted(int(x) for x in nd["RunningJobs"]) == sorted(np.nonzero(run)[0].tolist())


# ---- protobuf ---------------------------------------------------------------------------------
def test_cluster_state_bytes():
    # field 1 float 0.5 -> 0d 0000003f; field 2 float 0.25 -> 15 0000803e; optional field 3 = 160 ->
    # 18 a001; field 4 = 120000 -> 20 c0a907 (120000 = 0x1d4c0: 0x40|0x80, 0x29|0x80, 0x07); field 5
    # double 0 is omitted (implicit presence)
    assert W.marshal(W.cluster_state(0.5, 0.25, 0.0, totals=(160, 120000))).hex() == "0d0000003f150000803e18a00120c0a907"
    assert W.marshal(W.ClusterState()) == b""
    assert W.marshal(W.ClusterState(total_cpu=0)) == b"\x18\x00"        # optional: present when set
    assert W.marshal(W.ClusterState(cores_utilization=-0.0)).hex() == "0d00000080"  # -0.0 is not zero bits
    assert W.marshal(W.ClusterState(average_wait_time=600000.5)) == b"\x29" + struct.pack("<d", 600000.5)


def test_contract_and_node_messages():
    # ContractRequest{cores 33, memory 1, time 50 s, trader "x"}: 10 21 | 18 01 | 22 02 (08 32) | 32 01 78
    req = W.ContractRequest(cores=33, memory=1, time=W.Duration(50, 0), trader="x")
    assert W.marshal(req).hex() == "1021180122020832320178"
    assert W.unmarshal(W.ContractRequest, W.marshal(req)) == req
    resp = W.ContractResponse(id=4, approve=True, cores=2, memory=3, time=W.Duration(1, 5), price=1.5, trader="t")
    assert W.unmarshal(W.ContractResponse, W.marshal(resp)) == resp
    node = W.NodeObject(id=1, url="u", cores=2, memory=3, time=W.Duration(-1, -500))
    assert W.unmarshal(W.NodeObject, W.marshal(node)) == node
    # Duration{-1, -500}: int64/int32 negatives are 10-byte sign-extended varints
    assert W.marshal(W.Duration(-1, -500)).hex() == "08ffffffffffffffffff01108cfcffffffffffffff01"
    vn = W.VirtualNodeRequest(id=9, cores=1, memory=2, time=W.Duration.from_ns(-1_500_000_000))
    assert vn.time == W.Duration(-1, -500_000_000) and vn.time.to_ns() == -1_500_000_000
    assert W.unmarshal(W.VirtualNodeRequest, W.marshal(vn)) == vn


def test_provide_jobs_padding_d9():
    l1 = [(i + 1, 2 * i + 1, 3 * i) for i in range(21)]
    batches = W.provide_jobs_batches(l1)
    assert len(batches) == 2
    last = W.marshal(batches[1])
    # the 21st job {cores 21, mem 41, time 60 s}: 0a 08 | 08 15 10 29 1a 02 08 3c, then 19 nil
    # entries, each an empty Job message 0a 00
    assert last.hex() == "0a08081510291a02083c" + "0a00" * 19
    got = W.unmarshal(W.ProvideJobsResponse, last)
    assert len(got.jobs) == 20 and got.jobs[1] == W.PbJob()  # the trader sees zero jobs, not nil
    assert got.jobs[1].unix_time_seconds is None  # AsDuration(nil) = 0
    # a zero-duration job keeps a present, empty Duration (durationpb.New(0) is non-nil): 1a 00
    assert W.marshal(W.provide_jobs_batches([(1, 1, 0)])[0]).startswith(bytes.fromhex("0a06080110011a00"))


def test_unmarshal_skips_unknown_and_rejects_malformed():
    known = W.marshal(W.ContractRequest(id=5))
    extra = bytes.fromhex("f80101") + bytes.fromhex("1d00000000")  # field 31 varint; field 3 as fixed32
    assert W.unmarshal(W.ContractRequest, known + extra) == W.ContractRequest(id=5)
    # a message field seen twice merges (proto semantics)
    two = bytes.fromhex("22020832") + bytes.fromhex("22021005")
    assert W.unmarshal(W.ContractRequest, two).time == W.Duration(50, 5)
    for bad in (b"\x08", b"\x0d\x00\x00", b"\x32\x05ab", b"\x32\x01\xff", b"\x00\x01", b"\x0b"):
        with pytest.raises(W.WireError):
            W.unmarshal(W.ContractRequest, bad)
    # uint32 fields truncate wider varints like protobuf-go's uint32(v)
    assert W.unmarshal(W.ContractRequest, b"\x08" + bytes.fromhex("8180808010")).id == 1
