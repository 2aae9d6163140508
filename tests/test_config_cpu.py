"""Cluster-config loader (mochi_config_*) on the reference's own properties file.

tests/golden/sample_config is a byte copy of the reference's config/sample_config
(the file MochiDB boots from with -DclusterConfig); the loader must read it the
way ClusterConfiguration.loadInitialConfigurationFromProperties does
(ClusterConfiguration.java:138-187) and reproduce getServerMajority (:264-267)
and getServersForObject (:194-226, including the :215 token-index bug)."""
import os

import pytest

import mochi_hip as mh

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAMPLE = os.path.join(ROOT, "tests", "golden", "sample_config")

IDS = ["server-ed25bc93-1047-4242-b87b-2246355b020b", "server-55a78d3f-783d-43ae-95c1-6d0f5f02fe0c",
       "server-6c023c90-87ed-40d9-8f38-48cb03fa2135", "server-6a3b63b2-9fc8-4f3d-97c1-0f61cb244a0c",
       "server-20d27225-0253-4013-8f6c-b32afb3e5452"]


def ring(ids, n=1024):
    """putTokensAroundRingProps (ClusterConfiguration.java:89-118): round robin."""
    lines = []
    for s, sid in enumerate(ids):
        lines.append(f"_CONFIG_SERVER_{sid}_TOKENS=" + ",".join(str(t) for t in range(s, n, len(ids))))
        lines.append(f"_CONFIG_SERVER_{sid}_URL=127.0.0.1:{8001 + s}")
    return lines


def test_sample_config_r4():
    cfg = mh.ClusterConfig(SAMPLE)
    assert cfg.replication_factor == 4
    assert cfg.majority == 3 == mh.majority(4)
    servers = cfg.servers()
    assert [s for s, _ in servers] == IDS  # _CONFIG_SERVERS order
    assert dict(servers)[IDS[0]] == "127.0.0.1:8001" and dict(servers)[IDS[4]] == "127.0.0.1:8005"
    # tokens 0..3 belong to the first four servers (round robin): every key's replicas
    for key in ["DEMO_KEY_1", "DEMO_READ_KEY_2", "DEMO_KEY_STRESS_TEST_117", "", "ключ"]:
        assert cfg.servers_for_key(key) == [0, 1, 2, 3]
    assert cfg.replica_id_list() == IDS[:4]
    assert cfg.replica_id_list("DEMO_KEY_2") == IDS[:4]
    cfg.close()


def test_replica_table_feeds_the_workload():
    import workload as W

    assert W.SERVER_IDS[:4] == mh.ClusterConfig(SAMPLE).replica_id_list()


def test_properties_syntax():
    # comments, ':' separator, blanks around '=', continuation lines, escapes, last duplicate wins
    text = "\n".join([
        "# a comment", "! another", "   ",
        "_CONFIG_SERVERS : a,,b,\\", "    c,d",
        "_CONFIG_BFT_REPLICATION = 3", "_CONFIG_BFT_REPLICATION=4",
    ] + ring(["a", "b", "c", "d"]) + ["_CONFIG_SERVER_\\u0061_URL=host\\tA"])
    cfg = mh.ClusterConfig(text=text)
    assert cfg.replication_factor == 4 and cfg.majority == 3
    assert cfg.servers() == [("a", "host\tA"), ("b", "127.0.0.1:8002"), ("c", "127.0.0.1:8003"),
                             ("d", "127.0.0.1:8004")]
    assert cfg.replica_id_list() == ["a", "b", "c", "d"]


def test_ids_reach_the_wire_as_java_would_encode_them():
    """Properties.load(InputStream) reads ISO-8859-1: a raw byte >= 0x80 is one
    char (2 bytes of UTF-8 on the wire); \\uXXXX escapes are UTF-16 code units, a
    surrogate pair one supplementary char (4 bytes), a lone surrogate '?'
    (String.getBytes(UTF_8), protobuf-java's fallback)."""
    ids = [b"caf\xe9", b"s\\uD83D\\uDE00", b"lone\\uD800x", b"d"]
    lines = [b"_CONFIG_SERVERS=" + b",".join(ids), b"_CONFIG_BFT_REPLICATION=4"]
    for s, sid in enumerate(ids):
        lines.append(b"_CONFIG_SERVER_" + sid + b"_TOKENS=" + ",".join(str(t) for t in range(s, 1024, 4)).encode())
        lines.append(b"_CONFIG_SERVER_" + sid + b"_URL=127.0.0.1:" + str(8001 + s).encode())
    cfg = mh.ClusterConfig(text=b"\n".join(lines))
    want = ["caf\u00e9", "s\U0001F600", "lone?x", "d"]
    assert [s for s, _ in cfg.servers()] == want
    assert cfg.replica_id_list() == want
    blob, off = cfg.replica_ids()
    assert bytes(blob[off[1]:off[2]]) == "s\U0001F600".encode() and off[2] - off[1] == 5
    cfg.close()


def test_str_text_round_trips_ids():
    """ClusterConfig(text=str) writes the str the way Properties.store
    would (ISO-8859-1, \\uXXXX above U+00FF), so the ids read back as the same str
    -- not as its UTF-8 bytes re-read as Latin-1 ('caf\u00c3\u00a9')."""
    ids = ["caf\u00e9", "s\U0001F600", "\u4e2d", "d"]
    lines = ["_CONFIG_SERVERS=" + ",".join(ids), "_CONFIG_BFT_REPLICATION=4"]
    for s, sid in enumerate(ids):
        lines.append(f"_CONFIG_SERVER_{sid}_TOKENS=" + ",".join(str(t) for t in range(s, 1024, 4)))
        lines.append(f"_CONFIG_SERVER_{sid}_URL=127.0.0.1:{8001 + s}")
    cfg = mh.ClusterConfig(text="\n".join(lines))
    assert [s for s, _ in cfg.servers()] == ids
    assert cfg.replica_id_list() == ids
    cfg.close()


def test_r7_majority():
    ids = [f"s{i}" for i in range(8)]
    cfg = mh.ClusterConfig(text="\n".join(["_CONFIG_SERVERS=" + ",".join(ids), "_CONFIG_BFT_REPLICATION=7"]
                                          + ring(ids)))
    assert cfg.replication_factor == 7 and cfg.majority == 5
    assert cfg.servers_for_key("k") == list(range(7))


@pytest.mark.parametrize("case,msg", [
    ("r3", "should be > 4"),
    ("no_r", "non defined"),
    ("no_url", "Missing server url"),
    ("dup_token", "Mutple mapping"),
    ("big_token", "Too large shard number"),
    ("hole", "is not assigned"),
    ("bad_int", "For input string"),
])
def test_reference_errors(case, msg):
    ids = ["a", "b", "c", "d"]
    lines = ["_CONFIG_SERVERS=a,b,c,d", "_CONFIG_BFT_REPLICATION=4"] + ring(ids)
    if case == "r3":
        lines[1] = "_CONFIG_BFT_REPLICATION=3"
    elif case == "no_r":
        lines.pop(1)
    elif case == "no_url":
        lines = [x for x in lines if x != "_CONFIG_SERVER_c_URL=127.0.0.1:8003"]
    elif case == "dup_token":
        lines.append("_CONFIG_SERVER_d_TOKENS=" + ",".join(str(t) for t in range(3, 1024, 4)) + ",0")
    elif case == "big_token":
        lines.append("_CONFIG_SERVER_d_TOKENS=" + ",".join(str(t) for t in range(3, 1024, 4)) + ",1024")
    elif case == "hole":
        lines.append("_CONFIG_SERVER_d_TOKENS=" + ",".join(str(t) for t in range(7, 1024, 4)))
    elif case == "bad_int":
        lines[1] = "_CONFIG_BFT_REPLICATION=four"
    with pytest.raises(mh.MochiError, match=msg):
        mh.ClusterConfig(text="\n".join(lines))


def test_collision_when_r_exceeds_the_owners_of_tokens_0_to_r_minus_1():
    # 5 servers, R = 6: load passes (:183 compares R with the token count), the lookup throws (:217-222)
    cfg = mh.ClusterConfig(text="\n".join(["_CONFIG_SERVERS=" + ",".join(IDS), "_CONFIG_BFT_REPLICATION=6"] + ring(IDS)))
    with pytest.raises(mh.MochiError, match="unique"):
        cfg.servers_for_key("k")
