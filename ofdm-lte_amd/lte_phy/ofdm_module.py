"""OFDMModule facade (drop-in for the reference's ofdm_module.py:32-207): a
SISO OFDMSimulator with the backward-compatible API."""
from .config import LTEConfig
from .ofdm_core import OFDMSimulator


class OFDMModule:
    def __init__(self, config=None, channel_type='awgn', mode='lte', enable_sc_fdm=False,
                 enable_equalization=True):
        if config is None:
            config = LTEConfig()
        self.config, self.channel_type, self.mode = config, channel_type, mode
        self.enable_sc_fdm, self.enable_equalization = enable_sc_fdm, enable_equalization
        self.simulator = OFDMSimulator(config=config, channel_type=channel_type, mode=mode,
                                       enable_sc_fdm=enable_sc_fdm, enable_equalization=enable_equalization,
                                       num_channels=1)
        self.last_results = None

    def transmit(self, bits, snr_db=10.0):
        self.last_results = self.simulator.simulate_siso(bits, snr_db=snr_db)
        return self.last_results

    def _calculate_papr(self, signal):
        return self.simulator.tx.calculate_papr(signal)

    @property
    def channel(self):
        return self.simulator.channels[0]

    @property
    def modulator(self):
        return self.simulator.tx.modulator

    @property
    def demodulator(self):
        return self.simulator.rx.demodulator

    @property
    def tx(self):
        return self.simulator.tx

    @property
    def rx(self):
        return self.simulator.rx

    def run_ber_sweep(self, num_bits, snr_range, num_trials=1, progress_callback=None):
        return self.simulator.run_ber_sweep(num_bits, snr_range, num_trials=num_trials,
                                            progress_callback=progress_callback)

    def get_config(self):
        return self.config

    def __repr__(self):
        mode = "SC-FDM" if self.enable_sc_fdm else "OFDM"
        return f"OFDMModule({self.config.modulation}, {mode}, {self.channel_type})"
