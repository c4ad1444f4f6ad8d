"""Barra_factor_cal/config.py constants (same names and values; paths from MFA_* env vars)."""
import os

from llm_driven_multi_factor_model_amd.models.factor_engine import BARRA_OUTPUT_COLUMNS as _COLS
from llm_driven_multi_factor_model_amd.models.factor_engine import BARRA_RENAME as _RENAME
from llm_driven_multi_factor_model_amd.models.factor_engine import FACTORS_TO_RUN as _FACTORS
from llm_driven_multi_factor_model_amd.utils.config import FactorConfig as _FC

BASE_DIR = os.environ.get("MFA_BASE_DIR", os.path.dirname(os.path.abspath(__file__)))
DATA_DIR = os.environ.get("MFA_DATA_DIR", os.path.join(BASE_DIR, "data"))
RESULT_DIR = os.environ.get("MFA_RESULT_DIR", os.path.join(BASE_DIR, "result"))

STK_DATA_PATH = os.path.join(DATA_DIR, "csi300_stk_data_financial_index_balance_cashflow.csv")
INDEX_DATA_PATH = os.path.join(DATA_DIR, "csi_300_index_20200101_20250930.csv")
INDUSTRY_DATA_PATH = os.path.join(DATA_DIR, "stk_sw_industry.csv")

FACTORS_TO_RUN = list(_FACTORS)
COMPOSITE_CONFIG = _FC().composite
ORTHO_RULES = _FC().ortho
COLUMN_RENAME_MAP = dict(_RENAME)
BARRA_OUTPUT_COLUMNS = list(_COLS)

MONGO_CONNECTION_STRING = os.environ.get("MFA_MONGO_URI", "mongodb://localhost:27017/")
DB_NAME = os.environ.get("MFA_MONGO_DB", "barra_financial_data")
