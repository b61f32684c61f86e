"""Machine-learning-utility evaluator.

Output-compatible with ``real_res`` (`Server/utility_analysis.py:15-91`): categorical
columns are label-encoded with encoders fitted on ``original_real`` (train union test),
features are standardised with a scaler fitted on ``original_real``, and four classifiers
— logistic regression, decision tree and random forest (``class_weight="balanced",
random_state=69``) and an MLP (``random_state=69``) — are trained on ``real`` and scored
on ``test`` by accuracy and weighted F1.  The CLI prints the real-minus-synthetic
difference matrix and its mean F1 difference (`:114-119`).
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import pandas as pd


def real_res(original_real: pd.DataFrame, real: pd.DataFrame, test: pd.DataFrame, target_col: str,
             cat_cols: Sequence[str], verbose: bool = True) -> List[List[float]]:
    from sklearn import ensemble, linear_model, metrics, preprocessing, tree
    from sklearn.neural_network import MLPClassifier

    real, test, original_real = real.copy(), test.copy(), original_real.copy()
    for x in cat_cols or []:
        le = preprocessing.LabelEncoder()
        real[x] = real[x].astype(str)
        test[x] = test[x].astype(str)
        original_real[x] = original_real[x].astype(str)
        le.fit(original_real[x].values)
        real[x] = le.transform(real[x])
        test[x] = le.transform(test[x])
        original_real[x] = le.transform(original_real[x])
    y_tr, X_tr = real[target_col], real.drop(columns=[target_col])
    y_te, X_te = test[target_col], test.drop(columns=[target_col])
    scaler = preprocessing.StandardScaler().fit(original_real.drop(columns=[target_col]).values)
    Xs_tr, Xs_te = scaler.transform(X_tr.values), scaler.transform(X_te.values)
    models = [
        ("LR", lambda: linear_model.LogisticRegression(class_weight="balanced", random_state=69)),
        ("DT", lambda: tree.DecisionTreeClassifier(class_weight="balanced", random_state=69)),
        ("RF", lambda: ensemble.RandomForestClassifier(class_weight="balanced", random_state=69)),
        ("MLP", lambda: MLPClassifier(random_state=69)),
    ]
    out = []
    for name, make in models:
        if verbose:
            print(f"training of {name}")
        m = make().fit(Xs_tr, y_tr)
        pred = m.predict(Xs_te)
        out.append([metrics.accuracy_score(y_te, pred), metrics.f1_score(y_te, pred, average="weighted")])
    return out


def utility_difference(train: pd.DataFrame, test: pd.DataFrame, fake: pd.DataFrame, target_col: str,
                       cat_cols: Sequence[str], verbose: bool = True):
    original = pd.concat([train, test])
    r = real_res(original, train, test, target_col, cat_cols, verbose)
    f = real_res(original, fake, test, target_col, cat_cols, verbose)
    diff = np.asarray(r) - np.asarray(f)
    return diff, float(diff.mean(axis=0)[1])
