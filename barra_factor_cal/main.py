"""main.py compatibility: load -> descriptors -> post-process -> Barra export -> Mongo / CSV."""
from __future__ import annotations

import os

import pandas as pd

from llm_driven_multi_factor_model_amd.models.factor_engine import factor_pipeline

from . import config
from .load_data import load_and_prepare_data


def save_df_to_mongodb(db, df: pd.DataFrame, collection_name: str):
    if df.empty:
        print(f"Warning: DataFrame for collection '{collection_name}' is empty. Nothing to save.")
        return
    collection = db[collection_name]
    try:
        collection.drop()
        records = df.to_dict("records")
        collection.insert_many(records)
        print(f"Successfully saved {len(records)} records to '{collection_name}'.")
    except Exception as e:  # reference: log and continue (main.py:38-39)
        print(f"An error occurred while saving to '{collection_name}': {e}")


def main(db=None, csv_dir: str | None = None):
    stk, idx, sw = load_and_prepare_data(db)
    final, info, timings = factor_pipeline(stk, idx, sw)
    print(f"timings: {timings}")
    if csv_dir:
        os.makedirs(csv_dir, exist_ok=True)
        final.to_csv(os.path.join(csv_dir, "barra_data_csi.csv"), index=False)
        info.to_csv(os.path.join(csv_dir, "industry_info.csv"), index=False)
    target = db
    client = None
    if target is None:
        try:
            from pymongo import MongoClient
            client = MongoClient(config.MONGO_CONNECTION_STRING)
            target = client[config.DB_NAME]
        except Exception as e:
            print(f"\nFailed to connect to MongoDB to save results: {e}")
            return final, info
    save_df_to_mongodb(target, final, "barra_factors")
    save_df_to_mongodb(target, info, "sw_industry_info_for_factors")
    if client is not None:
        client.close()
    return final, info


if __name__ == "__main__":
    main(csv_dir=config.RESULT_DIR)
