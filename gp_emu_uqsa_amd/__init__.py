"""gp_emu_uqsa_amd -- MI355X-native hot path of the GP_emu_UQSA emulator."""
