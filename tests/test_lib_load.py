"""The library loader's source check (CPU: loading the library makes no GPU call).

A library built from other sources is refused; ``TK_LIB_PATH`` + ``TK_LIB_ANY_SOURCES=1`` (the
same-box A/B of two source versions in tools/) is the one way past the check, and only with the
path override.
"""
import pytest

from tachikoma_amd import _lib
import tachikoma_amd.build as build


@pytest.fixture
def fresh_loader(monkeypatch):
    saved = _lib._LIB
    _lib._LIB = None
    monkeypatch.setattr(build, "source_hash", lambda: "0" * 16)  # the tree "changed"
    yield
    _lib._LIB = saved


def test_other_sources_refused(fresh_loader, monkeypatch):
    monkeypatch.delenv("TK_LIB_PATH", raising=False)
    monkeypatch.setenv("TK_LIB_ANY_SOURCES", "1")  # ignored without the path override
    with pytest.raises(_lib.TachikomaError, match="built from other sources"):
        _lib.load()


def test_any_sources_needs_override_and_flag(fresh_loader, monkeypatch):
    monkeypatch.setenv("TK_LIB_PATH", _lib.LIB_PATH)
    monkeypatch.delenv("TK_LIB_ANY_SOURCES", raising=False)
    with pytest.raises(_lib.TachikomaError, match="built from other sources"):
        _lib.load()
    monkeypatch.setenv("TK_LIB_ANY_SOURCES", "1")
    lib = _lib.load()
    assert lib.tk_build_info().decode()
