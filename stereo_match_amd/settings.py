"""Settings handling mirrored from the reference CLI.

``parse_config_file`` follows ``disparity_calculation.py:75-128`` (same
defaults at ``:87-92``, same ``[disparity]`` keys and casts, a missing or
``None`` file returns the defaults).  Two optional extension keys select the
engine's north-star mode: ``cost`` (``"sgbm"`` | ``"census"``) and ``paths``
(5 = OpenCV MODE_SGBM, 8 = MODE_HH / 8-path).
"""
from __future__ import annotations

import configparser
import os

DEFAULT_SETTINGS = {
    'npz_file': '/media/hao/DATA/Arkit/05122017-105828/src/tmp.npz',
    'mode': 'P',
    'window_size': 3, 'min_disparity': 0, 'num_disparities': 160, 'block_size': 5, 'disp12_max_diff': 1,
    'uniqueness_ratio': 15, 'speckle_window_size': 0, 'speckle_range': 2, 'pre_filter_cap': 63,
    'lmbda': 80000, 'sigma': 1.2}

_INT_KEYS = ('window_size', 'min_disparity', 'num_disparities', 'block_size', 'disp12_max_diff',
             'uniqueness_ratio', 'speckle_window_size', 'speckle_range', 'pre_filter_cap', 'lmbda', 'paths')
_STR_KEYS = ('npz_file', 'mode', 'cost')


def parse_config_file(settings_file):
    """Parse a settings.ini ``[disparity]`` section (reference :75-128)."""
    settings = dict(DEFAULT_SETTINGS)
    if settings_file is None or not os.path.isfile(settings_file):
        return settings
    config = configparser.ConfigParser()
    config.read(settings_file)
    section = config['disparity']
    for key in _STR_KEYS:
        if key in section:
            settings[key] = str(section[key])
    for key in _INT_KEYS:
        if key in section:
            settings[key] = int(section[key])
    if 'sigma' in section:
        settings['sigma'] = float(section['sigma'])
    return settings
