"""Alias of the reference's root package (`from module import OFDMModule,
LTEConfig`, examples/example_basic.py:17) -> lte_phy.  `module.config`,
`module.core.*`, ... resolve to the sibling aliases in this directory."""
import os as _os

from _boot import PKG as _PKG  # noqa: F401
from lte_phy import *  # noqa: F401,F403
from lte_phy import __all__, OFDMModule, LTEConfig  # noqa: F401

__path__ = [_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))]
