"""LTE numerology (drop-in for the reference's config.py:1-215).

Same public names, constructor arguments, derived attributes and error
behaviour as `LTEConfig` (config.py:63-199); the tables are the reference's
LTE profile / CP / ITU-R M.1225 values.
"""
import numpy as np

LTE_PROFILES = {1.25: {'Nc': 76, 'N': 128}, 2.5: {'Nc': 150, 'N': 256}, 5.0: {'Nc': 300, 'N': 512},
                10.0: {'Nc': 600, 'N': 1024}, 15.0: {'Nc': 900, 'N': 2048}, 20.0: {'Nc': 1200, 'N': 2048}}
CP_VALUES = {'normal': 4.7, 'extended_15khz': 16.6, 'extended_7.5khz': 33.0}   # microseconds
MODULATION_SCHEMES = ['QPSK', '16-QAM', '64-QAM']
SUBCARRIER_SPACING = [15.0, 7.5]
ITU_CHANNEL_MODELS = {
    'Pedestrian_A': {'delays_us': [0.0, 0.11, 0.19, 0.41], 'power_db': [0.0, -9.7, -19.2, -22.8],
                     'description': 'Pedestrian, low velocity, short distance'},
    'Pedestrian_B': {'delays_us': [0.0, 0.2, 0.8, 1.2, 2.3, 3.7], 'power_db': [0.0, -0.9, -4.9, -8.0, -7.8, -23.9],
                     'description': 'Pedestrian, high velocity'},
    'Vehicular_A': {'delays_us': [0.0, 0.31, 0.71, 1.09, 1.73, 2.51],
                    'power_db': [0.0, -1.0, -9.0, -10.0, -15.0, -20.0],
                    'description': 'Vehicular, low velocity, short distance'},
    'Vehicular_B': {'delays_us': [0.0, 0.3, 0.7, 1.09, 1.73, 2.51, 3.7, 4.53],
                    'power_db': [0.0, -1.0, -9.0, -10.0, -13.0, -16.0, -21.6, -24.0],
                    'description': 'Vehicular, high velocity, long distance'},
    'Bad_Urban': {'delays_us': [0.0, 0.1, 0.3, 0.5, 0.9, 1.3, 1.9, 2.6],
                  'power_db': [0.0, -3.0, -5.0, -7.0, -9.0, -11.0, -13.0, -15.0],
                  'description': 'Urban with severe multipath'},
}
_BPS = {'QPSK': 2, '16-QAM': 4, '64-QAM': 6}


class LTEConfig:
    """LTE OFDM configuration; derives N, Nc, fs, CP length, bits/symbol."""

    def __init__(self, bandwidth=5.0, delta_f=15.0, modulation='QPSK', cp_type='normal'):
        self.bandwidth = bandwidth
        self.delta_f = delta_f
        self.modulation = modulation
        self.cp_type = cp_type
        if modulation not in MODULATION_SCHEMES:
            raise ValueError(f"Unsupported modulation: {modulation}. Options: {MODULATION_SCHEMES}")
        self._calculate_parameters()

    def _calculate_parameters(self):
        prof = LTE_PROFILES.get(self.bandwidth)
        if prof is not None:
            self.Nc, self.N = prof['Nc'], prof['N']
        else:
            self.Nc = int((self.bandwidth * 1e3) / self.delta_f)
            self.N = self._next_power_of_2(self.Nc)
        self.fs = self.N * self.delta_f * 1e3
        self.Ts = 1 / self.fs
        self.T_symbol = self.N * self.Ts
        self.cp_duration = self._get_cp_duration()
        self.cp_length = int(self.cp_duration * 1e-6 * self.fs)
        self.bits_per_symbol = self._get_bits_per_symbol()
        self.samples_per_ofdm_symbol = self.N + self.cp_length

    @staticmethod
    def _next_power_of_2(x):
        return int(2 ** np.ceil(np.log2(x)))

    def _get_cp_duration(self):
        if self.cp_type == 'extended':
            return CP_VALUES['extended_15khz'] if self.delta_f == 15.0 else CP_VALUES['extended_7.5khz']
        return CP_VALUES['normal']

    def _get_bits_per_symbol(self):
        return _BPS.get(self.modulation, 2)

    def get_info(self):
        return {'Bandwidth (MHz)': self.bandwidth, 'Subcarrier Spacing (kHz)': self.delta_f,
                'Modulation': self.modulation, 'CP Type': self.cp_type, 'Useful Subcarriers (Nc)': self.Nc,
                'FFT Points (N)': self.N, 'Sampling Frequency (MHz)': self.fs / 1e6,
                'Sampling Period (ns)': self.Ts * 1e9, 'OFDM Symbol Duration (μs)': self.T_symbol * 1e6,
                'CP Duration (μs)': self.cp_duration, 'CP Length (samples)': self.cp_length,
                'Bits per Symbol': self.bits_per_symbol, 'Samples per OFDM Symbol': self.samples_per_ofdm_symbol}

    def __str__(self):
        return "\n".join(["LTE OFDM Configuration:"] + [f"  {k}: {v}" for k, v in self.get_info().items()])

    def __repr__(self):
        return (f"LTEConfig(bandwidth={self.bandwidth}, delta_f={self.delta_f}, "
                f"modulation='{self.modulation}', cp_type='{self.cp_type}')")

    def copy(self):
        return LTEConfig(self.bandwidth, self.delta_f, self.modulation, self.cp_type)


def create_config_5MHz_QPSK():
    return LTEConfig(bandwidth=5.0, delta_f=15.0, modulation='QPSK', cp_type='normal')


def create_config_20MHz_16QAM():
    return LTEConfig(bandwidth=20.0, delta_f=15.0, modulation='16-QAM', cp_type='normal')


def create_config_10MHz_64QAM():
    return LTEConfig(bandwidth=10.0, delta_f=15.0, modulation='64-QAM', cp_type='normal')
