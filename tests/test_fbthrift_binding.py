"""The fbthrift-side binding of GpuBatchSerializer.h (THRIFT_GPU_WITH_FBTHRIFT):
every reference name that mode uses must be declared by a header that mode
includes, transitively, in the reference tree.

libthriftcpp2 cannot be built in this image (folly, fmt, glog, gflags and
boost are absent), so the mode cannot be compiled here; this test is the
declaration check instead (round-4 verdict, "Missing 1"):

* every `#include <thrift/...>` of the block exists under /root/reference;
* every `apache::thrift::...` name the block uses is *defined* (class /
  struct / enum with a body, not only forward-declared) in one of the
  headers those includes reach, inside the right namespace;
* the TProtocolException constructor and enum the block calls exist with the
  argument list used;
* folly is not vendored in the reference: `folly::IOBuf` / `IOBufQueue` are
  checked to come from the same headers the reference's protocols include
  (`BinaryProtocol.h:21-22`), and every member the batch templates call on
  them (with the arity used) is called the same way by the reference's own
  code.

A negative control re-runs the resolution with the CompactV1 include removed
(the round-4 defect) and requires it to fail. Skips when /root/reference is
absent (the GPU box)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
HDR = os.path.join(ROOT, "include", "thrift_gpu", "GpuBatchSerializer.h")

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "thrift")),
                                reason="reference tree absent")


def fbthrift_blocks(text):
    """The text of every `#ifdef THRIFT_GPU_WITH_FBTHRIFT` branch (up to its
    #else / #endif; the header's blocks do not nest)."""
    out, on = [], False
    for line in text.splitlines():
        s = line.strip()
        if s.startswith("#ifdef THRIFT_GPU_WITH_FBTHRIFT"):
            on = True
            continue
        if on and (s.startswith("#else") or s.startswith("#endif")):
            on = False
            continue
        if on:
            out.append(line)
    return "\n".join(out)


def include_closure(includes):
    """Reference headers reachable from `includes` through thrift/ includes."""
    seen, todo = set(), list(includes)
    while todo:
        inc = todo.pop()
        path = os.path.join(REF, inc)
        if path in seen or not os.path.isfile(path):
            continue
        seen.add(path)
        with open(path, errors="replace") as f:
            for m in re.finditer(r'#include\s+[<"](thrift/[^>"]+)[>"]', f.read()):
                todo.append(m.group(1))
    return seen


def defined_in(closure, ns, name):
    """Files of the closure defining `name` (with a body) in namespace `ns`."""
    body = re.compile(r"\b(class|struct|enum)\s+(?:FOLLY_EXPORT\s+)?%s\b[^;{]*\{" % re.escape(name))
    nsre = re.compile(r"namespace\s+%s\s*\{|namespace\s+%s\s*\{" % (
        re.escape(ns), r"\s*\{\s*namespace\s+".join(map(re.escape, ns.split("::")))))
    hits = []
    for p in closure:
        with open(p, errors="replace") as f:
            t = f.read()
        if body.search(t) and nsre.search(t):
            hits.append(p)
    return hits


def resolve(block):
    """[(name, ok, where)] for every reference name the block uses."""
    incs = re.findall(r"#include\s+<([^>]+)>", block)
    thrift_incs = [i for i in incs if i.startswith("thrift/")]
    closure = include_closure(thrift_incs)
    names = sorted(set(re.findall(r"apache::thrift::(?:\w+::)*\w+", block)))
    res = []
    for q in names:
        parts = q.split("::")
        name, ns = parts[-1], "::".join(parts[:-1])
        hits = defined_in(closure, ns, name)
        res.append((q, bool(hits), hits[:1]))
    return incs, thrift_incs, closure, res


def test_block_includes_exist():
    block = fbthrift_blocks(open(HDR).read())
    incs, thrift_incs, closure, _ = resolve(block)
    assert thrift_incs, "the fbthrift block includes no thrift headers"
    for i in thrift_incs:
        assert os.path.isfile(os.path.join(REF, i)), i
    # the three protocol headers the tags name, and the exception's
    for need in ("thrift/lib/cpp2/protocol/BinaryProtocol.h",
                 "thrift/lib/cpp2/protocol/CompactProtocol.h",
                 "thrift/lib/cpp2/protocol/CompactV1Protocol.h",
                 "thrift/lib/cpp/protocol/TProtocolException.h"):
        assert os.path.join(REF, need) in closure, need


def test_every_reference_name_resolves():
    block = fbthrift_blocks(open(HDR).read())
    _, _, _, res = resolve(block)
    names = [q for q, _, _ in res]
    for expect in ("apache::thrift::BinaryProtocolReader", "apache::thrift::BinaryProtocolWriter",
                   "apache::thrift::CompactProtocolReader", "apache::thrift::CompactProtocolWriter",
                   "apache::thrift::CompactV1ProtocolReader",
                   "apache::thrift::CompactV1ProtocolWriter",
                   "apache::thrift::protocol::TProtocolException"):
        assert expect in names, expect
    bad = [q for q, ok, _ in res if not ok]
    assert not bad, "names without a definition in the included headers: %s" % bad


def test_exception_interface_matches():
    """makeProtocolException calls TProtocolException(TProtocolExceptionType,
    const std::string&) and casts to TProtocolException::TProtocolExceptionType
    (TProtocolException.h:41-51,62-63)."""
    block = fbthrift_blocks(open(HDR).read())
    assert "TProtocolException::TProtocolExceptionType" in block
    t = open(os.path.join(REF, "thrift/lib/cpp/protocol/TProtocolException.h")).read()
    assert re.search(r"enum\s+TProtocolExceptionType\s*\{", t)
    assert re.search(r"TProtocolException\(\s*TProtocolExceptionType\s+\w+,\s*const std::string&", t)
    # the type codes the C ABI reports (tgpu_status.tproto_type) are the enum's
    codes = dict(re.findall(r"\b([A-Z_]+)\s*=\s*(\d+),", t.split("enum TProtocolExceptionType")[1]
                            .split("}")[0]))
    assert codes == {"UNKNOWN": "0", "INVALID_DATA": "1", "NEGATIVE_SIZE": "2", "SIZE_LIMIT": "3",
                     "BAD_VERSION": "4", "NOT_IMPLEMENTED": "5", "MISSING_REQUIRED_FIELD": "6",
                     "CHECKSUM_MISMATCH": "7", "DEPTH_LIMIT": "8"}


def _ref_calls(pattern):
    """Whether the reference's own cpp2 code has a line matching `pattern`."""
    rx = re.compile(pattern)
    base = os.path.join(REF, "thrift", "lib", "cpp2")
    for d, _, files in os.walk(base):
        for fn in files:
            if not fn.endswith((".h", ".cpp")):
                continue
            with open(os.path.join(d, fn), errors="replace") as f:
                for line in f:
                    if rx.search(line):
                        return True
    return False


def test_folly_members_used_as_the_reference_uses_them():
    text = open(HDR).read()
    block = fbthrift_blocks(text)
    assert "#include <folly/io/IOBuf.h>" in block and "#include <folly/io/IOBufQueue.h>" in block
    bp = open(os.path.join(REF, "thrift/lib/cpp2/protocol/BinaryProtocol.h")).read()
    assert "#include <folly/io/IOBuf.h>" in bp and "#include <folly/io/IOBufQueue.h>" in bp
    # the members the batch templates call on IOBuf / IOBufQueue (outside the
    # stand-in classes), with the arity used there
    body = text[text.index("std::vector<uint8_t> coalesced("):]
    used = {
        "isChained": r"->isChained\(\)",
        "data": r"->data\(\)",
        "length": r"->length\(\)",
        "computeChainDataLength": r"->computeChainDataLength\(\)",
        "next": r"->next\(\)",
        "preallocate2": r"->preallocate\(\w+, \w+\)",
        "postallocate": r"->postallocate\(\w+\)",
    }
    ref = {
        "isChained": r"\bisChained\(\)",
        "data": r"\bbuf->data\(\)|\biobuf->data\(\)",
        "length": r"\bbuf->length\(\)",
        "computeChainDataLength": r"computeChainDataLength\(\)",
        "next": r"->next\(\)",
        "preallocate2": r"\bpreallocate\(\s*[\w.]+,\s*[\w.]+\)",
        "postallocate": r"\bpostallocate\(\w+\)",
    }
    for k, rx in used.items():
        assert re.search(rx, body), "batch code no longer calls %s" % k
        assert _ref_calls(ref[k]), "the reference never calls %s this way" % k


def test_negative_control_catches_missing_include():
    """Without the CompactV1 include (round 4's header) the CompactV1 tags do
    not resolve."""
    block = fbthrift_blocks(open(HDR).read())
    broken = block.replace("#include <thrift/lib/cpp2/protocol/CompactV1Protocol.h>", "")
    assert broken != block
    _, _, _, res = resolve(broken)
    bad = {q for q, ok, _ in res if not ok}
    assert bad == {"apache::thrift::CompactV1ProtocolReader",
                   "apache::thrift::CompactV1ProtocolWriter"}, bad
