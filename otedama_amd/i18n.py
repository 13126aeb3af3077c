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
        STARTUP_WALLET_CREATED: "已创建新的闪电网络钱包,其恢复种子已加密保存在本机。",
        STARTUP_HARDWARE_FOUND: "发现 {{.count}} 台挖矿设备:{{.summary}}",
        STARTUP_HARDWARE_NONE: "未检测到挖矿设备。Otedama 需要 MI355X GPU 或受支持的 CPU。",
        STARTUP_POOL_CONNECTING: "正在连接矿池 {{.url}}...",
        STARTUP_POOL_CONNECTED: "已连接矿池 {{.url}}。",
        ERROR_POOL_UNREACHABLE: "无法连接矿池 {{.url}}。请检查网络或配置其他矿池。",
        ERROR_INVALID_ADDRESS: "比特币地址 {{.address}} 无效,请检查是否有输入错误。",
        ERROR_CONFIG_MISSING: "开始挖矿前需要比特币地址。请使用 --bitcoin-address 或设置 OTEDAMA_BITCOIN_ADDRESS。",
        ERROR_WALLET_LOCKED: "闪电网络钱包已锁定。请输入密码短语解锁后继续。",
        ERROR_HARDWARE_FAILURE: "设备 {{.id}} 报告硬件故障,已停止使用。",
        STATUS_MINING: "正在 {{.devices}} 台设备上挖矿。当前算力:{{.hashrate}}。",
        STATUS_IDLE: "空闲:矿池当前没有分配工作。",
        STATUS_PAYMENT_RECEIVED: "已从矿池 {{.pool}} 收到 {{.amount}}。",
        STATUS_SHUTTING_DOWN: "正在安全退出。您的钱包仍安全保存在本机。",
    },
    "ko": {
        STARTUP_READY: "Otedama 준비 완료. 곧 채굴을 시작합니다.",
        STARTUP_WALLET_CREATED: "새 라이트닝 지갑을 만들었습니다. 복구 시드는 이 장치에 암호화되어 저장됩니다.",
        STARTUP_HARDWARE_FOUND: "채굴 장치 {{.count}}대를 찾았습니다: {{.summary}}",
        STARTUP_HARDWARE_NONE: "채굴 장치를 찾지 못했습니다. MI355X GPU 또는 지원되는 CPU가 필요합니다.",
        STARTUP_POOL_CONNECTING: "풀 {{.url}}에 연결하는 중...",
        STARTUP_POOL_CONNECTED: "풀 {{.url}}에 연결되었습니다.",
        ERROR_POOL_UNREACHABLE: "풀 {{.url}}에 연결할 수 없습니다. 네트워크를 확인하거나 다른 풀을 설정하세요.",
        ERROR_INVALID_ADDRESS: "비트코인 주소 {{.address}}가 올바르지 않습니다. 오타가 없는지 확인하세요.",
        ERROR_CONFIG_MISSING: "채굴을 시작하려면 비트코인 주소가 필요합니다. --bitcoin-address 를 지정하거나 "
                              "OTEDAMA_BITCOIN_ADDRESS 를 설정하세요.",
        ERROR_WALLET_LOCKED: "라이트닝 지갑이 잠겨 있습니다. 암호 문구로 잠금을 해제하세요.",
        ERROR_HARDWARE_FAILURE: "장치 {{.id}}에서 하드웨어 오류가 발생하여 사용을 중지했습니다.",
        STATUS_MINING: "{{.devices}}대 장치에서 채굴 중. 현재 해시레이트: {{.hashrate}}.",
        STATUS_IDLE: "대기 중: 지금은 풀에서 받은 작업이 없습니다.",
        STATUS_PAYMENT_RECEIVED: "풀 {{.pool}}에서 {{.amount}}을(를) 받았습니다.",
        STATUS_SHUTTING_DOWN: "안전하게 종료하는 중입니다. 지갑은 이 장치에 안전하게 보관됩니다.",
    },
    "es": {
        STARTUP_READY: "Otedama está listo. La minería comenzará en breve.",
        STARTUP_WALLET_CREATED: "Se creó un nuevo monedero Lightning; su semilla de recuperación se guarda cifrada en "
                                "este equipo.",
        STARTUP_HARDWARE_FOUND: "Se encontraron {{.count}} dispositivo(s) de minería: {{.summary}}",
        STARTUP_HARDWARE_NONE: "No se detectaron dispositivos de minería. Otedama necesita una GPU MI355X o una CPU "
                               "compatible.",
        STARTUP_POOL_CONNECTING: "Conectando al pool {{.url}}...",
        STARTUP_POOL_CONNECTED: "Conectado al pool {{.url}}.",
        ERROR_POOL_UNREACHABLE: "No se puede alcanzar el pool {{.url}}. Revisa la red o configura otro pool.",
        ERROR_INVALID_ADDRESS: "La dirección Bitcoin {{.address}} no es válida. Revisa si hay errores de escritura.",
        ERROR_CONFIG_MISSING: "Se necesita una dirección Bitcoin para empezar a minar. Usa --bitcoin-address o define "
                              "OTEDAMA_BITCOIN_ADDRESS.",
        ERROR_WALLET_LOCKED: "El monedero Lightning está bloqueado. Desbloquéalo con tu frase de contraseña.",
        ERROR_HARDWARE_FAILURE: "El dispositivo {{.id}} informó un fallo de hardware y se retiró del servicio.",
        STATUS_MINING: "Minando en {{.devices}} dispositivo(s). Hashrate actual: {{.hashrate}}.",
        STATUS_IDLE: "En espera: el pool no tiene trabajo para nosotros ahora mismo.",
        STATUS_PAYMENT_RECEIVED: "Se recibieron {{.amount}} del pool {{.pool}}.",
        STATUS_SHUTTING_DOWN: "Cerrando de forma segura. Tu monedero sigue protegido en este equipo.",
    },
    "fr": {
        STARTUP_READY: "Otedama est prêt. Le minage va commencer.",
        STARTUP_WALLET_CREATED: "Un nouveau portefeuille Lightning a été créé ; sa graine de récupération est "
                                "chiffrée sur cet appareil.",
        STARTUP_HARDWARE_FOUND: "{{.count}} appareil(s) de minage trouvé(s) : {{.summary}}",
        STARTUP_HARDWARE_NONE: "Aucun appareil de minage détecté. Otedama nécessite un GPU MI355X ou un CPU pris en "
                               "charge.",
        STARTUP_POOL_CONNECTING: "Connexion au pool {{.url}}...",
        STARTUP_POOL_CONNECTED: "Connecté au pool {{.url}}.",
        ERROR_POOL_UNREACHABLE: "Le pool {{.url}} est injoignable. Vérifiez le réseau ou configurez un autre pool.",
        ERROR_INVALID_ADDRESS: "L'adresse Bitcoin {{.address}} n'est pas valide. Vérifiez les fautes de frappe.",
        ERROR_CONFIG_MISSING: "Une adresse Bitcoin est requise pour commencer. Utilisez --bitcoin-address ou "
                              "définissez OTEDAMA_BITCOIN_ADDRESS.",
        ERROR_WALLET_LOCKED: "Le portefeuille Lightning est verrouillé. Déverrouillez-le avec votre phrase secrète.",
        ERROR_HARDWARE_FAILURE: "L'appareil {{.id}} a signalé une panne matérielle et a été mis hors service.",
        STATUS_MINING: "Minage sur {{.devices}} appareil(s). Hashrate actuel : {{.hashrate}}.",
        STATUS_IDLE: "En attente : le pool n'a pas de travail pour nous pour le moment.",
        STATUS_PAYMENT_RECEIVED: "{{.amount}} reçu(s) du pool {{.pool}}.",
        STATUS_SHUTTING_DOWN: "Arrêt en cours. Votre portefeuille reste en sécurité sur cet appareil.",
    },
    "de": {
        STARTUP_READY: "Otedama ist bereit. Das Mining beginnt in Kürze.",
        STARTUP_WALLET_CREATED: "Eine neue Lightning-Wallet wurde erstellt; ihr Wiederherstellungs-Seed liegt "
                                "verschlüsselt auf diesem Gerät.",
        STARTUP_HARDWARE_FOUND: "{{.count}} Mining-Gerät(e) gefunden: {{.summary}}",
        STARTUP_HARDWARE_NONE: "Keine Mining-Geräte erkannt. Otedama benötigt eine MI355X-GPU oder eine unterstützte "
                               "CPU.",
        STARTUP_POOL_CONNECTING: "Verbinde mit Pool {{.url}}...",
        STARTUP_POOL_CONNECTED: "Mit Pool {{.url}} verbunden.",
        ERROR_POOL_UNREACHABLE: "Pool {{.url}} ist nicht erreichbar. Prüfen Sie das Netzwerk oder richten Sie einen "
                                "anderen Pool ein.",
        ERROR_INVALID_ADDRESS: "Die Bitcoin-Adresse {{.address}} ist ungültig. Bitte auf Tippfehler prüfen.",
        ERROR_CONFIG_MISSING: "Zum Starten wird eine Bitcoin-Adresse benötigt. Verwenden Sie --bitcoin-address oder "
                              "setzen Sie OTEDAMA_BITCOIN_ADDRESS.",
        ERROR_WALLET_LOCKED: "Die Lightning-Wallet ist gesperrt. Entsperren Sie sie mit Ihrer Passphrase.",
        ERROR_HARDWARE_FAILURE: "Gerät {{.id}} hat einen Hardwarefehler gemeldet und wurde außer Betrieb genommen.",
        STATUS_MINING: "Mining auf {{.devices}} Gerät(en). Aktuelle Hashrate: {{.hashrate}}.",
        STATUS_IDLE: "Leerlauf: Der Pool hat gerade keine Arbeit für uns.",
        STATUS_PAYMENT_RECEIVED: "{{.amount}} vom Pool {{.pool}} erhalten.",
        STATUS_SHUTTING_DOWN: "Wird sauber beendet. Ihre Wallet bleibt sicher auf diesem Gerät.",
    },
    "pt": {
        STARTUP_READY: "O Otedama está pronto. A mineração começará em breve.",
        STARTUP_WALLET_CREATED: "Uma nova carteira Lightning foi criada; a semente de recuperação fica cifrada neste "
                                "dispositivo.",
        STARTUP_HARDWARE_FOUND: "{{.count}} dispositivo(s) de mineração encontrado(s): {{.summary}}",
        STARTUP_HARDWARE_NONE: "Nenhum dispositivo de mineração detectado. O Otedama precisa de uma GPU MI355X ou de "
                               "uma CPU compatível.",
        STARTUP_POOL_CONNECTING: "Conectando ao pool {{.url}}...",
        STARTUP_POOL_CONNECTED: "Conectado ao pool {{.url}}.",
        ERROR_POOL_UNREACHABLE: "O pool {{.url}} está inacessível. Verifique a rede ou configure outro pool.",
        ERROR_INVALID_ADDRESS: "O endereço Bitcoin {{.address}} é inválido. Verifique se há erros de digitação.",
        ERROR_CONFIG_MISSING: "É necessário um endereço Bitcoin para começar a minerar. Use --bitcoin-address ou "
                              "defina OTEDAMA_BITCOIN_ADDRESS.",
        ERROR_WALLET_LOCKED: "A carteira Lightning está bloqueada. Desbloqueie-a com sua frase-senha.",
        ERROR_HARDWARE_FAILURE: "O dispositivo {{.id}} relatou uma falha de hardware e foi retirado de serviço.",
        STATUS_MINING: "Minerando em {{.devices}} dispositivo(s). Hashrate atual: {{.hashrate}}.",
        STATUS_IDLE: "Ocioso: o pool não tem trabalho para nós no momento.",
        STATUS_PAYMENT_RECEIVED: "Recebido {{.amount}} do pool {{.pool}}.",
        STATUS_SHUTTING_DOWN: "Encerrando com segurança. Sua carteira continua protegida neste dispositivo.",
    },
    "ru": {
        STARTUP_READY: "Otedama готова. Майнинг скоро начнётся.",
        STARTUP_WALLET_CREATED: "Создан новый Lightning-кошелёк; его seed для восстановления хранится на этом "
                                "устройстве в зашифрованном виде.",
        STARTUP_HARDWARE_FOUND: "Найдено устройств для майнинга: {{.count}} ({{.summary}})",
        STARTUP_HARDWARE_NONE: "Устройства для майнинга не найдены. Нужен GPU MI355X или поддерживаемый CPU.",
        STARTUP_POOL_CONNECTING: "Подключение к пулу {{.url}}...",
        STARTUP_POOL_CONNECTED: "Подключено к пулу {{.url}}.",
        ERROR_POOL_UNREACHABLE: "Пул {{.url}} недоступен. Проверьте сеть или настройте другой пул.",
        ERROR_INVALID_ADDRESS: "Биткоин-адрес {{.address}} недействителен. Проверьте, нет ли опечаток.",
        ERROR_CONFIG_MISSING: "Для начала майнинга нужен биткоин-адрес. Укажите --bitcoin-address или задайте "
                              "OTEDAMA_BITCOIN_ADDRESS.",
        ERROR_WALLET_LOCKED: "Lightning-кошелёк заблокирован. Разблокируйте его своей парольной фразой.",
        ERROR_HARDWARE_FAILURE: "Устройство {{.id}} сообщило об аппаратной ошибке и выведено из работы.",
        STATUS_MINING: "Майнинг на {{.devices}} устройствах. Текущий хешрейт: {{.hashrate}}.",
        STATUS_IDLE: "Ожидание: у пула сейчас нет для нас работы.",
        STATUS_PAYMENT_RECEIVED: "Получено {{.amount}} от пула {{.pool}}.",
        STATUS_SHUTTING_DOWN: "Корректное завершение. Ваш кошелёк остаётся в безопасности на этом устройстве.",
    },
    "ar": {
        STARTUP_READY: "Otedama جاهز. سيبدأ التعدين قريبًا.",
        STARTUP_WALLET_CREATED: "تم إنشاء محفظة Lightning جديدة؛ بذرة الاسترداد محفوظة مشفّرة على هذا الجهاز.",
        STARTUP_HARDWARE_FOUND: "تم العثور على {{.count}} جهاز تعدين: {{.summary}}",
        STARTUP_HARDWARE_NONE: "لم يتم اكتشاف أجهزة تعدين. يحتاج Otedama إلى وحدة MI355X أو معالج مدعوم.",
        STARTUP_POOL_CONNECTING: "جارٍ الاتصال بالمجمّع {{.url}}...",
        STARTUP_POOL_CONNECTED: "تم الاتصال بالمجمّع {{.url}}.",
        ERROR_POOL_UNREACHABLE: "تعذّر الوصول إلى المجمّع {{.url}}. تحقق من الشبكة أو اضبط مجمّعًا آخر.",
        ERROR_INVALID_ADDRESS: "عنوان البيتكوين {{.address}} غير صالح. تحقق من عدم وجود أخطاء كتابية.",
        ERROR_CONFIG_MISSING: "يلزم عنوان بيتكوين لبدء التعدين. استخدم --bitcoin-address أو اضبط "
                              "OTEDAMA_BITCOIN_ADDRESS.",
        ERROR_WALLET_LOCKED: "محفظة Lightning مقفلة. افتحها باستخدام عبارة المرور.",
        ERROR_HARDWARE_FAILURE: "أبلغ الجهاز {{.id}} عن عطل في العتاد وتم إيقافه عن العمل.",
        STATUS_MINING: "التعدين على {{.devices}} جهاز. معدل التجزئة الحالي: {{.hashrate}}.",
        STATUS_IDLE: "خامل: لا يوجد عمل من المجمّع حاليًا.",
        STATUS_PAYMENT_RECEIVED: "تم استلام {{.amount}} من المجمّع {{.pool}}.",
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
