"""The Scala FFM binding and its C++ transcription (FfmMirror, tests/cpp/test_ffm_sequence.cpp,
which the GPU tests run) must not drift apart: per method, the same native calls in the same order,
and the rsv_config offsets FfmSampler writes must be the C struct's (CPU only; no JDK needed).

No JDK exists in this image, so the Scala cannot be compiled here; this is the check that the GPU
evidence about FfmMirror still speaks for FfmSampler.scala."""
import ctypes as C
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCALA = os.path.join(ROOT, "bindings", "scala", "ffm", "lgbt", "princess", "reservoir", "gpu", "ffm", "FfmSampler.scala")
MIRROR = os.path.join(ROOT, "tests", "cpp", "test_ffm_sequence.cpp")


def _body(src: str, header: str) -> str:
    """Text of the brace block that follows `header` (first occurrence)."""
    i = src.index(header)
    j = src.index("{", i + len(header) - 1)
    depth = 0
    for p in range(j, len(src)):
        depth += {"{": 1, "}": -1}.get(src[p], 0)
        if depth == 0:
            return src[j:p + 1]
    raise ValueError(header)


def _snake(name: str) -> str:
    return re.sub(r"(?<!^)(?=[A-Z])", "_", name).lower()


def _scala_calls(body: str) -> list:
    out = []
    for m in re.finditer(r"\b(rsv[A-Z]\w*)\.invoke|\b(nextStage)\(\)|\b(cleanable)\.clean\(\)", body):
        if m.group(1):
            out.append(_snake(m.group(1)))
        elif m.group(2):
            out.append("next_stage")
        else:
            out.append("rsv_destroy")  # the Cleaner action: rsvDestroy + arena close
    return out


def _cpp_calls(body: str) -> list:
    return [m.group(1) for m in re.finditer(r"\b(rsv_(?!jvm)\w+|next_stage)\(", body)]


def test_ffm_mirror_call_sequences_match_scala():
    scala = open(SCALA).read()
    cpp = open(MIRROR).read()
    mirror = _body(cpp, "struct FfmMirror {")
    pairs = [("private[this] def nextStage(): Unit = {", "void next_stage() {"),
             ("def sample(element: A): Unit = {", "void sample(const void* key, int64_t hash) {"),
             ("def result(): IndexedSeq[B] = {", "std::vector<uint8_t> result(int64_t* n_out) {"),
             ("override def sampleAll(elements: IterableOnce[A]): Unit = elements match {",
              "int64_t sample_all_indexed(int64_t n, KeyAt key_at) {")]
    for s_head, c_head in pairs:
        s_calls = _scala_calls(_body(scala, s_head))
        c_calls = _cpp_calls(_body(mirror, c_head))
        assert s_calls and s_calls == c_calls, (s_head, s_calls, c_calls)
    # construction: rsv_config_init + rsv_create in Scala; the harness inits the config before it
    ctor = _scala_calls(_body(scala, "private[this] val handle: MemorySegment = {"))
    assert ctor == ["rsv_config_init", "rsv_create"], ctor
    assert "rsv_create(" in _body(mirror, "FfmMirror(const rsv_config& c)")


def test_ffm_config_offsets_match_c_struct():
    from reservoir_amd._native import RsvConfig

    scala = open(SCALA).read()
    body = _body(scala, "private[this] val handle: MemorySegment = {")
    names = {"kind": "kind", "maxSampleSize": "max_sample_size", "keys.width": "key_width",
             "if (reusable) 1 else 0": "reusable", "engine": "engine", "hashKind": "hash_kind", "seed": "seed"}
    sets = [m.groups() for m in (re.match(r"\s*cfg\.set\((JAVA_INT|JAVA_LONG), (\d+)L, (.*)\)\s*$", ln)
                                  for ln in body.splitlines()) if m]
    assert len(sets) == len(names), sets
    for layout, off, expr in sets:
        field = names[expr.strip()]
        assert getattr(RsvConfig, field).offset == int(off), (field, off)
        size = 8 if layout == "JAVA_LONG" else 4
        assert getattr(RsvConfig, field).size == size, field
    # the StructLayout's field order = the C struct's
    layout = re.findall(r'JAVA_(?:INT|LONG)\.withName\("(\w+)"\)', scala)
    assert layout == [f for f, _ in RsvConfig._fields_], layout
    assert C.sizeof(RsvConfig) == 56
