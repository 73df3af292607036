"""Locations of the in-tree native libraries (built by the package Makefile)."""
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))


def lib_path(name: str) -> str:
    p = os.path.join(PKG_DIR, name)
    if not os.path.exists(p):
        raise FileNotFoundError(
            f"{name} is not built: run `make -C {os.path.dirname(PKG_DIR)}` "
            "(or __graft_entry__.build())")
    return p
