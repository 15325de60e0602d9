"""HPACK codec (RFC 7541): Appendix C vectors + property tests."""
from hypothesis import given, settings, strategies as st


def test_huffman_rfc_c4_vectors(n):
    # RFC 7541 C.4.1 - C.4.3 Huffman-coded header values
    vectors = {
        "www.example.com": "f1e3c2e5f23a6ba0ab90f4ff",
        "no-cache": "a8eb10649cbf",
        "custom-key": "25a849e95ba97d7f",
        "custom-value": "25a849e95bb8e8b4bf",
    }
    for s, hx in vectors.items():
        assert n.hpack_huffman_encode(s).hex() == hx
        assert n.hpack_huffman_decode(bytes.fromhex(hx)) == s.encode()


def test_huffman_rejects_bad_padding(n):
    good = bytes.fromhex("a8eb10649cbf")
    assert n.hpack_huffman_decode(good[:-1] + bytes([good[-1] & 0xFE])) is None  # padding not all ones
    assert n.hpack_huffman_decode(good + b"\xff") is None  # >= 8 bits of padding


@settings(max_examples=300, deadline=None)
@given(st.binary(max_size=200))
def test_huffman_roundtrip(n, data):
    enc = n.hpack_huffman_encode(data)
    assert n.hpack_huffman_decode(enc) == data


def test_rfc_c3_requests_without_huffman(n):
    d = n.HpackDecoder(4096)
    r1 = bytes.fromhex("828684410f7777772e6578616d706c652e636f6d")
    assert d.decode(r1) == [(":method", "GET"), (":scheme", "http"), (":path", "/"),
                            (":authority", "www.example.com")]
    assert d.table_size == 57
    r2 = bytes.fromhex("828684be58086e6f2d6361636865")
    assert d.decode(r2) == [(":method", "GET"), (":scheme", "http"), (":path", "/"),
                            (":authority", "www.example.com"), ("cache-control", "no-cache")]
    assert d.table_size == 110
    r3 = bytes.fromhex("828785bf400a637573746f6d2d6b65790c637573746f6d2d76616c7565")
    assert d.decode(r3) == [(":method", "GET"), (":scheme", "https"), (":path", "/index.html"),
                            (":authority", "www.example.com"), ("custom-key", "custom-value")]
    assert d.table_size == 164 and d.table_entries == 3


def test_rfc_c4_requests_with_huffman(n):
    d = n.HpackDecoder(4096)
    assert d.decode(bytes.fromhex("828684418cf1e3c2e5f23a6ba0ab90f4ff"))[3] == (":authority", "www.example.com")
    assert d.decode(bytes.fromhex("828684be5886a8eb10649cbf"))[4] == ("cache-control", "no-cache")
    out = d.decode(bytes.fromhex("828785bf408825a849e95ba97d7f8925a849e95bb8e8b4bf"))
    assert out[-1] == ("custom-key", "custom-value") and d.table_size == 164


def test_rfc_c5_responses_with_eviction(n):
    d = n.HpackDecoder(256)
    # C.5.1: dynamic table size 256 -> entries are evicted across the three responses
    r1 = bytes.fromhex("4803333032580770726976617465611d4d6f6e2c203231204f637420323031332032303a31333a323120474d"
                       "546e1768747470733a2f2f7777772e6578616d706c652e636f6d")
    assert d.decode(r1)[0] == (":status", "302") and d.table_size == 222
    r2 = bytes.fromhex("4803333037c1c0bf")
    assert d.decode(r2)[0] == (":status", "307") and d.table_size == 222


def test_decoder_errors(n):
    d = n.HpackDecoder(4096)
    assert d.decode(bytes([0x80])) is None          # index 0
    assert d.decode(bytes([0xBF])) is None          # index 63: empty dynamic table
    assert d.decode(bytes([0x3F, 0xE2, 0x1F])) is None  # size update 4097 > advertised 4096
    assert d.decode(bytes([0x3F, 0xE1, 0x1F])) == []    # exactly 4096 is allowed
    assert d.decode(bytes([0x82, 0x20])) is None    # size update after a header


def test_integer_prefix_examples(n):
    # RFC C.1: 1337 with a 5-bit prefix = 1f 9a 0a; via a literal name length we can check
    d = n.HpackDecoder(8192)
    name = "a" * 1337
    block = b"\x00" + bytes([0x7F, 0xBA, 0x09]) + name.encode() + b"\x01x"  # 127 + 1210 = 1337 (7-bit prefix)
    assert d.decode(block) == [(name, "x")]


@settings(max_examples=500, deadline=None)
@given(st.binary(max_size=64))
def test_table_huffman_decoder_matches_bitwise_reference(n, blob):
    """Arbitrary bytes (mostly invalid codes/padding): the table-driven decoder used on
    the request path accepts and rejects exactly what the bit-by-bit decoder does."""
    assert n.hpack_huffman_decode(blob) == n.hpack_huffman_decode_bitwise(blob)


@settings(max_examples=300, deadline=None)
@given(st.binary(max_size=300))
def test_table_huffman_decoder_roundtrip_long_codes(n, data):
    enc = n.hpack_huffman_encode(data)  # bytes >= 0x80 use the long (> 10 bit) codes
    assert n.hpack_huffman_decode(enc) == data == n.hpack_huffman_decode_bitwise(enc)


def test_visitor_decode_matches_vector_decode(n):
    """The server's non-allocating decode keeps the same dynamic-table state and yields
    the same headers as the vector decode, across RFC C.3-C.5 sequences (incl. eviction)."""
    seqs = [(4096, ["828684410f7777772e6578616d706c652e636f6d", "828684be58086e6f2d6361636865",
                    "828785bf400a637573746f6d2d6b65790c637573746f6d2d76616c7565"]),
            (4096, ["828684418cf1e3c2e5f23a6ba0ab90f4ff", "828684be5886a8eb10649cbf",
                    "828785bf408825a849e95ba97d7f8925a849e95bb8e8b4bf"]),
            (256, ["4803333032580770726976617465611d4d6f6e2c203231204f637420323031332032303a31333a323120474d"
                   "546e1768747470733a2f2f7777772e6578616d706c652e636f6d", "4803333037c1c0bf"])]
    for size, blocks in seqs:
        a, b = n.HpackDecoder(size), n.HpackDecoder(size)
        for hx in blocks:
            assert a.decode(bytes.fromhex(hx)) == b.decode_visit(bytes.fromhex(hx))
            assert (a.table_size, a.table_entries) == (b.table_size, b.table_entries)
    d = n.HpackDecoder(64)  # an entry larger than the table is delivered and empties it
    big = b"\x40\x01a" + bytes([60]) + b"v" * 60
    assert d.decode_visit(big) == [("a", "v" * 60)] and d.table_entries == 0
    for bad in (b"\x80", b"\xbf", b"\x82\x20"):
        assert n.HpackDecoder(4096).decode_visit(bad) is None
