"""CPU: the image-transfer harness's host conversions (lte_phy/
image_processing.py ImageProcessor) against the
reference's own ImageProcessor outputs (tests/golden/golden_image.npz, made
from the reference's test image resized to 64x64).  Exact equality."""
import numpy as np
import pytest

from conftest import unpack

PIL = pytest.importorskip('PIL')


def test_image_bits_round_trip(golden_image):
    from PIL import Image
    from lte_phy.image_processing import ImageProcessor as IP
    g = golden_image
    img = Image.fromarray(g['img64'])
    bits, meta = IP.image_to_bits(img)
    assert np.array_equal(bits, unpack(g['img64_bits'], int(g['img64_nbits'][0])))
    assert (meta['height'], meta['width'], meta['channels']) == (64, 64, 3)
    assert np.array_equal(np.array(IP.bits_to_image(bits, meta)), g['img64'])


def test_corrupted_stream_and_psnr(golden_image):
    from PIL import Image
    from lte_phy.image_processing import ImageProcessor as IP
    g = golden_image
    img = Image.fromarray(g['img64'])
    bits, meta = IP.image_to_bits(img)
    flip = unpack(g['flip_bits'], len(bits))
    rec = IP.bits_to_image(flip, meta)
    assert np.array_equal(np.array(rec), g['flip_img'])
    assert [IP.calculate_psnr(img, rec), IP.calculate_psnr_bits(bits, flip), IP.calculate_psnr(img, img)] == \
        list(g['flip_psnr'])
    short = flip[:len(flip) - 1001]                     # short streams are zero-padded
    assert np.array_equal(np.array(IP.bits_to_image(short, meta)), g['short_img'])
    assert IP.calculate_psnr_bits(bits, short) == g['short_psnr_bits'][0]


def test_save_comparison(tmp_path, golden_image):
    from PIL import Image
    from lte_phy.image_processing import ImageProcessor as IP
    g = golden_image
    src = tmp_path / 'a.png'
    Image.fromarray(g['img64']).save(src)
    comp = IP.save_comparison(str(src), Image.fromarray(g['flip_img']), str(tmp_path / 'c.png'))
    assert comp.size == (128, 64)
    assert np.array_equal(np.array(comp)[:, 64:], g['flip_img'])
    assert IP.load_image_pil(str(src)).mode == 'RGB'
