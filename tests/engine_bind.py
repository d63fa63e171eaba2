"""Load the product package (directory `gossip-sim_amd/`, not an importable name)."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "gossip-sim_amd")


def load():
    if "gossip_sim_amd" in sys.modules:
        return sys.modules["gossip_sim_amd"]
    spec = importlib.util.spec_from_file_location("gossip_sim_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["gossip_sim_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


gs = load()
import gossip_sim_amd.synth as synth  # noqa: E402,F401
