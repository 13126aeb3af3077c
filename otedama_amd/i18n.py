"""Localised user-facing messages (10 priority languages).

Parity: internal/i18n/message.go (ID validation, Lang + 10 priority languages,
Catalog, Bundle.Render/RenderWith/MissingTranslations/Languages) and
internal/i18n/messages/{bundle,en,ja,...}.go (NewBundle, DetectLang with base
fallback, DetectLangFromEnv over LC_ALL/LC_MESSAGES/LANG with POSIX-locale
normalisation). Templates use ``{{.name}}`` placeholders like Go's
text/template; missing translations fall back to English.
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass

PRIORITY_LANGUAGES = ("en", "ja", "zh", "ko", "es", "fr", "de", "pt", "ru", "ar")
_ID_RE = re.compile(r"^[a-z0-9_.]+$")


class I18nError(ValueError):
    pass


def valid_id(s: str) -> bool:
    return bool(s) and s[0] != "." and s[-1] != "." and bool(_ID_RE.match(s))


STARTUP_READY = "startup.ready"
STARTUP_WALLET_CREATED = "startup.wallet_created"
STARTUP_HARDWARE_FOUND = "startup.hardware_found"
STARTUP_HARDWARE_NONE = "startup.hardware_none"
STARTUP_POOL_CONNECTING = "startup.pool_connecting"
STARTUP_POOL_CONNECTED = "startup.pool_connected"
ERROR_POOL_UNREACHABLE = "error.pool_unreachable"
ERROR_INVALID_ADDRESS = "error.invalid_address"
ERROR_CONFIG_MISSING = "error.config_missing"
ERROR_WALLET_LOCKED = "error.wallet_locked"
ERROR_HARDWARE_FAILURE = "error.hardware_failure"
STATUS_MINING = "status.mining"
STATUS_IDLE = "status.idle"
STATUS_PAYMENT_RECEIVED = "status.payment_received"
STATUS_SHUTTING_DOWN = "status.shutting_down"

ALL_IDS = tuple(sorted([
    STARTUP_READY, STARTUP_WALLET_CREATED, STARTUP_HARDWARE_FOUND, STARTUP_HARDWARE_NONE, STARTUP_POOL_CONNECTING,
    STARTUP_POOL_CONNECTED, ERROR_POOL_UNREACHABLE, ERROR_INVALID_ADDRESS, ERROR_CONFIG_MISSING, ERROR_WALLET_LOCKED,
    ERROR_HARDWARE_FAILURE, STATUS_MINING, STATUS_IDLE, STATUS_PAYMENT_RECEIVED, STATUS_SHUTTING_DOWN]))

_EN = {
    STARTUP_READY: "Otedama is ready. Mining will begin shortly.",
    STARTUP_WALLET_CREATED: "A new Lightning wallet was created; its recovery seed is kept encrypted on this device.",
    STARTUP_HARDWARE_FOUND: "Found {{.count}} mining device(s): {{.summary}}",
    STARTUP_HARDWARE_NONE: "No mining devices detected. Otedama needs an MI355X GPU or a supported CPU.",
    STARTUP_POOL_CONNECTING: "Connecting to pool {{.url}}...",
    STARTUP_POOL_CONNECTED: "Connected to pool {{.url}}.",
    ERROR_POOL_UNREACHABLE: "Pool {{.url}} is unreachable. Check the network or configure another pool.",
    ERROR_INVALID_ADDRESS: "Bitcoin address {{.address}} is not valid. Please check it for typos.",
    ERROR_CONFIG_MISSING: "A Bitcoin address is required before mining can start. Pass --bitcoin-address or set "
                          "OTEDAMA_BITCOIN_ADDRESS.",
    ERROR_WALLET_LOCKED: "The Lightning wallet is locked. Unlock it with your passphrase to continue.",
    ERROR_HARDWARE_FAILURE: "Device {{.id}} reported a hardware fault and was taken out of service.",
    STATUS_MINING: "Mining on {{.devices}} device(s). Current hashrate: {{.hashrate}}.",
    STATUS_IDLE: "Idle: the pool has no work for us right now.",
    STATUS_PAYMENT_RECEIVED: "Received {{.amount}} from pool {{.pool}}.",
    STATUS_SHUTTING_DOWN: "Shutting down cleanly. Your wallet stays safe on this device.",
}

_TRANSLATIONS: dict[str, dict[str, str]] = {
    "ja": {
        STARTUP_READY: "Otedamaの準備ができました。まもなくマイニングを開始します。",
        STARTUP_WALLET_CREATED: "新しいLightningウォレットを作成しました。復元シードはこの端末に暗号化して保存されています。",
        STARTUP_HARDWARE_FOUND: "マイニングデバイスを{{.count}}台検出しました: {{.summary}}",
        STARTUP_HARDWARE_NONE: "マイニングデバイスが見つかりません。MI355X GPUまたは対応CPUが必要です。",
        STARTUP_POOL_CONNECTING: "プール {{.url}} に接続しています...",
        STARTUP_POOL_CONNECTED: "プール {{.url}} に接続しました。",
        ERROR_POOL_UNREACHABLE: "プール {{.url}} に到達できません。ネットワークを確認するか別のプールを設定してください。",
        ERROR_INVALID_ADDRESS: "ビットコインアドレス {{.address}} が無効です。入力ミスがないか確認してください。",
        ERROR_CONFIG_MISSING: "マイニングを開始するにはビットコインアドレスが必要です。--bitcoin-address を指定するか "
                              "OTEDAMA_BITCOIN_ADDRESS を設定してください。",
        ERROR_WALLET_LOCKED: "Lightningウォレットがロックされています。パスフレーズで解除してください。",
        ERROR_HARDWARE_FAILURE: "デバイス {{.id}} でハードウェア障害が発生したため、使用を停止しました。",
        STATUS_MINING: "{{.devices}}台でマイニング中。現在のハッシュレート: {{.hashrate}}。",
        STATUS_IDLE: "待機中: 現在プールから作業がありません。",
        STATUS_PAYMENT_RECEIVED: "プール {{.pool}} から {{.amount}} を受け取りました。",
        STATUS_SHUTTING_DOWN: "安全に終了しています。ウォレットはこの端末に安全に保管されています。",
    },
    "zh": {
        STARTUP_READY: "Otedama 已就绪,即将开始挖矿。",
        STARTUP_POOL_CONNECTING: "正在连接矿池 {{.url}}...",
        STARTUP_POOL_CONNECTED: "已连接矿池 {{.url}}。",
        STARTUP_HARDWARE_FOUND: "发现 {{.count}} 台挖矿设备:{{.summary}}",
        ERROR_INVALID_ADDRESS: "比特币地址 {{.address}} 无效,请检查是否有输入错误。",
        STATUS_MINING: "正在 {{.devices}} 台设备上挖矿。当前算力:{{.hashrate}}。",
        STATUS_SHUTTING_DOWN: "正在安全退出。您的钱包仍安全保存在本机。",
    },
    "ko": {
        STARTUP_READY: "Otedama 준비 완료. 곧 채굴을 시작합니다.",
        STARTUP_POOL_CONNECTING: "풀 {{.url}}에 연결하는 중...",
        STARTUP_POOL_CONNECTED: "풀 {{.url}}에 연결되었습니다.",
        STATUS_MINING: "{{.devices}}대 장치에서 채굴 중. 현재 해시레이트: {{.hashrate}}.",
        STATUS_SHUTTING_DOWN: "안전하게 종료하는 중입니다. 지갑은 이 장치에 안전하게 보관됩니다.",
    },
    "es": {
        STARTUP_READY: "Otedama está listo. La minería comenzará en breve.",
        STARTUP_POOL_CONNECTING: "Conectando al pool {{.url}}...",
        STARTUP_POOL_CONNECTED: "Conectado al pool {{.url}}.",
        STATUS_MINING: "Minando en {{.devices}} dispositivo(s). Hashrate actual: {{.hashrate}}.",
        STATUS_SHUTTING_DOWN: "Cerrando de forma segura. Tu monedero sigue protegido en este equipo.",
    },
    "fr": {
        STARTUP_READY: "Otedama est prêt. Le minage va commencer.",
        STARTUP_POOL_CONNECTING: "Connexion au pool {{.url}}...",
        STATUS_SHUTTING_DOWN: "Arrêt en cours. Votre portefeuille reste en sécurité sur cet appareil.",
    },
    "de": {
        STARTUP_READY: "Otedama ist bereit. Das Mining beginnt in Kürze.",
        STARTUP_POOL_CONNECTING: "Verbinde mit Pool {{.url}}...",
        STATUS_SHUTTING_DOWN: "Wird sauber beendet. Ihre Wallet bleibt sicher auf diesem Gerät.",
    },
    "pt": {
        STARTUP_READY: "O Otedama está pronto. A mineração começará em breve.",
        STARTUP_POOL_CONNECTING: "Conectando ao pool {{.url}}...",
        STATUS_SHUTTING_DOWN: "Encerrando com segurança. Sua carteira continua protegida neste dispositivo.",
    },
    "ru": {
        STARTUP_READY: "Otedama готова. Майнинг скоро начнётся.",
        STARTUP_POOL_CONNECTING: "Подключение к пулу {{.url}}...",
        STATUS_SHUTTING_DOWN: "Корректное завершение. Ваш кошелёк остаётся в безопасности на этом устройстве.",
    },
    "ar": {
        STARTUP_READY: "Otedama جاهز. سيبدأ التعدين قريبًا.",
        STARTUP_POOL_CONNECTING: "جارٍ الاتصال بالمجمّع {{.url}}...",
        STATUS_SHUTTING_DOWN: "يتم الإيقاف بأمان. تبقى محفظتك آمنة على هذا الجهاز.",
    },
}


@dataclass
class Catalog:
    lang: str
    messages: dict[str, str]

    def __post_init__(self):
        if self.lang not in PRIORITY_LANGUAGES:
            raise I18nError(f"i18n: unsupported language {self.lang!r}")
        for k in self.messages:
            if not valid_id(k):
                raise I18nError(f"i18n: invalid message id {k!r}")


_PLACEHOLDER = re.compile(r"\{\{\s*\.(\w+)\s*\}\}")


class Bundle:
    def __init__(self, catalogs: list[Catalog]):
        self.catalogs = {c.lang: c for c in catalogs}
        if "en" not in self.catalogs:
            raise I18nError("i18n: bundle requires an English catalog")

    def languages(self) -> list[str]:
        return [lang for lang in PRIORITY_LANGUAGES if lang in self.catalogs]

    def render(self, lang: str, mid: str) -> str:
        return self.render_with(lang, mid, {})

    def render_with(self, lang: str, mid: str, data: dict | None = None) -> str:
        cat = self.catalogs.get(lang)
        tmpl = (cat.messages.get(mid) if cat else None) or self.catalogs["en"].messages.get(mid)
        if tmpl is None:
            raise I18nError(f"i18n: unknown message id {mid!r}")
        data = data or {}
        return _PLACEHOLDER.sub(lambda m: str(data.get(m.group(1), "<no value>")), tmpl)

    def missing_translations(self, lang: str) -> list[str]:
        cat = self.catalogs.get(lang)
        have = cat.messages if cat else {}
        return sorted(mid for mid in self.catalogs["en"].messages if mid not in have)


def new_bundle() -> Bundle:
    cats = [Catalog("en", dict(_EN))]
    cats += [Catalog(lang, dict(msgs)) for lang, msgs in _TRANSLATIONS.items()]
    return Bundle(cats)


def detect_lang(tag: str) -> str:
    if not tag:
        return "en"
    cand = tag.lower()
    if cand in PRIORITY_LANGUAGES:
        return cand
    base = re.split(r"[-_]", cand, maxsplit=1)[0]
    return base if base in PRIORITY_LANGUAGES else "en"


def _normalize_posix_locale(s: str) -> str:
    s = re.split(r"[.@]", s, maxsplit=1)[0]
    if s in ("", "C", "POSIX"):
        return ""
    return s.replace("_", "-")


def detect_lang_from_env(getenv=os.environ.get) -> str:
    for key in ("LC_ALL", "LC_MESSAGES", "LANG"):
        v = getenv(key) or ""
        if not v:
            continue
        tag = _normalize_posix_locale(v)
        return detect_lang(tag) if tag else "en"
    return "en"
