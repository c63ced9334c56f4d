"""Image transfer over the GPU link.

`ImageProcessor` is the drop-in for the reference's utils/image_processing.py
(:9-255): RGB image <-> MSB-first bit stream, PSNR from images or bit
streams, SSIM when scikit-image is present, side-by-side comparisons.  These
are host-side byte conversions around the chain.

`transmit_image` is the GUI / test "single" flow (SIMO/gui/main_window.py:
50-131, test/test_coded_image_comparison.py:135-330): image -> bits -> one
simulate_* call on the GPU (ref-compat randomness, identical to the
reference's own run) -> bits -> image -> PSNR / SSIM.

`transmit_payload` is the throughput form of the same: a real payload cut into
transport blocks that run as ONE batch of independent frames per GPU call
(Philox channel randomness per frame, lte_run), for payloads far larger than
the reference's one-frame-at-a-time flow.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import numpy as np

from . import _capi as C
from .ofdm_core import SLOT_SIZE, OFDMSimulator

try:
    from PIL import Image
except ImportError:  # pragma: no cover - Pillow is part of the reference's requirements
    Image = None


def _need_pil():
    if Image is None:
        raise ImportError("Pillow is required for the image harness (utils/image_processing.py imports PIL)")


class ImageProcessor:
    """utils/image_processing.py ImageProcessor (static methods)."""

    @staticmethod
    def _load(image):
        _need_pil()
        img = image if isinstance(image, Image.Image) else Image.open(image)
        return img.convert('RGB') if img.mode != 'RGB' else img

    @staticmethod
    def image_to_bits(image_path):
        """(:12-48) -> (bits uint8 [H*W*3*8], metadata)."""
        arr = np.array(ImageProcessor._load(image_path))
        h, w, c = arr.shape
        meta = {'height': h, 'width': w, 'channels': c, 'dtype': str(arr.dtype)}
        return np.unpackbits(arr.flatten()), meta

    @staticmethod
    def bits_to_image(bits, metadata):
        """(:50-89): zero-pad or truncate to H*W*C*8 bits, pack, reshape."""
        _need_pil()
        h, w, c = metadata['height'], metadata['width'], metadata['channels']
        need = h * w * c * 8
        bits = np.asarray(bits)
        bits = np.pad(bits, (0, need - len(bits)), 'constant') if len(bits) < need else bits[:need]
        flat = np.packbits(bits)
        try:
            return Image.fromarray(flat.reshape(h, w, c).astype(np.uint8), 'RGB')
        except Exception:
            return Image.new('RGB', (w, h), color='black')

    @staticmethod
    def calculate_psnr(original_img, reconstructed_img):
        """(:91-129) 20 log10(255 / sqrt(MSE)); inf for identical images."""
        a = np.array(original_img) if Image is not None and isinstance(original_img, Image.Image) else original_img
        b = np.array(reconstructed_img) if Image is not None and isinstance(reconstructed_img, Image.Image) \
            else reconstructed_img
        if a.shape != b.shape:
            b = np.array(Image.fromarray(b).resize((a.shape[1], a.shape[0])))
        mse = np.mean((a.astype(float) - b.astype(float)) ** 2)
        if mse == 0:
            return float('inf')
        return 20 * np.log10(255.0 / np.sqrt(mse))

    @staticmethod
    def calculate_psnr_bits(original_bits, reconstructed_bits):
        """(:131-168) PSNR of the byte streams the bit arrays pack into."""
        n = min(len(original_bits), len(reconstructed_bits))
        a, b = np.asarray(original_bits)[:n], np.asarray(reconstructed_bits)[:n]
        pad = (8 - n % 8) % 8
        if pad:
            a = np.concatenate([a, np.zeros(pad, dtype=int)])
            b = np.concatenate([b, np.zeros(pad, dtype=int)])
        mse = np.mean((np.packbits(a).astype(float) - np.packbits(b).astype(float)) ** 2)
        if mse == 0:
            return float('inf')
        return 20 * np.log10(255.0 / np.sqrt(mse))

    @staticmethod
    def calculate_ssim(original_img, reconstructed_img):
        """(:170-204): scikit-image SSIM, None when scikit-image is absent."""
        try:
            from skimage.metrics import structural_similarity as ssim
        except ImportError:
            print("scikit-image no disponible para calcular SSIM")
            return None
        a, b = np.array(original_img), np.array(reconstructed_img)
        if a.shape != b.shape:
            b = np.array(Image.fromarray(b).resize((a.shape[1], a.shape[0])))
        return ssim(a, b, channel_axis=2, data_range=255)

    @staticmethod
    def save_comparison(original_path, reconstructed_img, output_path):
        """(:206-233) side-by-side original | reconstructed."""
        orig = ImageProcessor._load(original_path)
        if orig.size != reconstructed_img.size:
            reconstructed_img = reconstructed_img.resize(orig.size)
        w, h = orig.size
        comp = Image.new('RGB', (w * 2, h))
        comp.paste(orig, (0, 0))
        comp.paste(reconstructed_img, (w, 0))
        comp.save(output_path)
        return comp

    @staticmethod
    def load_image_pil(image_path):
        """(:235-255)."""
        return ImageProcessor._load(image_path)


def transmit_image(image, simulator: OFDMSimulator, snr_db: float, mode: str = 'siso', num_rx: int = 2,
                   resize: Optional[tuple] = None) -> Dict:
    """One image through one simulate_* call (mode 'siso', 'simo', 'coded',
    'miso', 'mimo'); resize=(w, h) resamples with LANCZOS first, like the
    reference's coded image test.  Returns the simulate_* result plus
    'reconstructed_image', 'original_image', 'metadata', 'psnr', 'ssim'."""
    img = ImageProcessor._load(image)
    if resize is not None:
        img = img.resize(tuple(resize), Image.Resampling.LANCZOS)
    bits, meta = ImageProcessor.image_to_bits(img)
    bits = bits.astype(np.int64)
    if mode == 'siso':
        r = simulator.simulate_siso(bits, snr_db=snr_db)
    elif mode == 'simo':
        r = simulator.simulate_simo(bits, snr_db=snr_db, num_rx=num_rx)
    elif mode == 'coded':
        r = simulator.simulate_siso_coded(bits, snr_db=snr_db)
    elif mode == 'miso':
        r = simulator.simulate_miso(bits, snr_db=snr_db)
    elif mode == 'mimo':
        r = simulator.simulate_mimo(bits, snr_db=snr_db, num_rx=num_rx)
    else:
        raise ValueError(f"unknown mode {mode!r}")
    rec = ImageProcessor.bits_to_image(r['bits_received_array'], meta)
    out = dict(r)
    out.update({'reconstructed_image': rec, 'original_image': img, 'metadata': meta,
                'psnr': ImageProcessor.calculate_psnr(img, rec), 'ssim': ImageProcessor.calculate_ssim(img, rec)})
    return out


def transmit_payload(bits, simulator: OFDMSimulator, snr_db: float, coded: bool = True,
                     tb_bits: Optional[int] = None, seed: int = 0, frames_per_call: int = 4096) -> Dict:
    """Real payload bits through the chain as a batch of independent frames:
    coded -> transport blocks of tb_bits (default 27760, the config-2 TB) with
    CRC-24A + turbo; uncoded -> one 14-symbol subframe of data REs per frame.
    The last frame is zero-padded.  Channel draws are Philox keyed by (seed,
    frame index).  Returns the received bits (trimmed), bit errors, BER and
    per-frame CRC flags (coded)."""
    bits = np.asarray(bits).astype(np.uint8) & 1
    if bits.size == 0:
        raise ValueError("Bits array cannot be empty")
    cfg = simulator.config
    if coded:
        nb = int(tb_bits or 27760)
        plan = simulator._plan(C.CHAIN_CODED, 0, nb, max_frames=frames_per_call)
    else:
        nb = int(tb_bits or SLOT_SIZE * simulator.Nd * cfg.bits_per_symbol)
        plan = simulator._plan(C.CHAIN_UNCODED, int(np.ceil(nb / (simulator.Nd * cfg.bits_per_symbol))), nb,
                               max_frames=frames_per_call)
    nf = -(-len(bits) // nb)
    frames = np.zeros((nf, nb), dtype=np.uint8)
    frames.reshape(-1)[:len(bits)] = bits
    rx = np.empty_like(frames)
    crc = np.ones(nf, dtype=np.uint8)
    for i in range(0, nf, frames_per_call):
        f = frames[i:i + frames_per_call]
        r = plan.run(np.full(len(f), snr_db, dtype=np.float64), seed=seed, frame_id0=i, bits=f,
                     capture=('bits_rx',))
        rx[i:i + len(f)] = r['bits_rx']
        if coded:
            crc[i:i + len(f)] = r['crc_ok']
    out = rx.reshape(-1)[:len(bits)]
    err = int(np.sum(out != bits))
    return {'bits_received_array': out, 'bit_errors': err, 'ber': err / len(bits), 'frames': nf,
            'crc_ok': crc if coded else None, 'tb_bits': nb}


__all__ = ['ImageProcessor', 'transmit_image', 'transmit_payload']
