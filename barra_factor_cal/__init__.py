"""Drop-in replacement for the reference ``Barra_factor_cal`` scripts (config, factor_calculator,
post_processing, load_data, main), backed by the MI355X engine.  The reference imports these as
top-level modules from its own directory; here they are ``barra_factor_cal.<module>``."""
