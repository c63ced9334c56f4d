"""Puts ofdm-lte_amd/ (the lte_phy package) on sys.path for the reference
module-name aliases in this directory."""
import os
import sys

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if PKG not in sys.path:
    sys.path.insert(0, PKG)
